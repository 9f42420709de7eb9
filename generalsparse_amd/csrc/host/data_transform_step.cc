// data_transform_step.cc -- flat-array implementations of the hot-path transforms.
// Each function cites the reference file it reproduces.
#include "data_transform_step.hpp"

#include <map>

#include <algorithm>
#include <numeric>

namespace gs {

void basic_data_transform_step::replace_u(POS_TYPE p, const char *n, std::vector<uint64_t> v) {
    if (meta_data_set_ptr->is_exist(p, n, target_matrix_id)) meta_data_set_ptr->remove_element(p, n, target_matrix_id);
    meta_data_set_ptr->add_element(p, n, target_matrix_id, std::make_shared<universal_array>(std::move(v)));
    dst(p, n);
}

void basic_data_transform_step::replace_f(POS_TYPE p, const char *n, std::vector<double> v, data_type t) {
    if (meta_data_set_ptr->is_exist(p, n, target_matrix_id)) meta_data_set_ptr->remove_element(p, n, target_matrix_id);
    meta_data_set_ptr->add_element(p, n, target_matrix_id, std::make_shared<universal_array>(std::move(v), t));
    dst(p, n);
}

static inline double padding_bound() { return (double)get_config().PADDING_RATE_UP_BOUND; }

// ------------------------------------------------------------------ sort
// get_row_order_by_length.cc:14-126: stable bucket sort by row length, longest first
void get_row_order_by_length::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    GS_CHECK(!m.is_exist(GLOBAL_META, "original_nz_row_indices", s), "get_row_order_by_length: already sorted");
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t minr = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t maxr = m.scalar(GLOBAL_META, "end_row_index", s);
    GS_CHECK(maxr >= minr, "end_row_index < begin_row_index");
    uint64_t real_max = row.back();
    if (real_max > maxr - minr) maxr = minr + real_max;
    uint64_t nrow = maxr - minr + 1;
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, nrow - 1, 0, row.size() - 1);
    uint64_t maxlen = *std::max_element(cnt.begin(), cnt.end());
    std::vector<uint64_t> off(maxlen + 1, 0);
    for (uint64_t c : cnt) off[c]++;
    uint64_t acc = 0;
    for (int64_t L = (int64_t)maxlen; L >= 0; L--) {
        uint64_t c = off[L];
        off[L] = acc;
        acc += c;
    }
    std::vector<uint64_t> order(nrow);
    for (uint64_t i = 0; i < nrow; i++) order[off[cnt[i]]++] = i;
    src(GLOBAL_META, "nz_row_indices");
    replace_u(GLOBAL_META, "original_nz_row_indices", std::move(order));
    is_run = true;
}

namespace {
// start offset of every old row in the row-sorted COO
std::vector<uint64_t> old_row_starts(const std::vector<uint64_t> &row, uint64_t nrow) {
    std::vector<uint64_t> start(nrow + 1, 0);
    for (uint64_t r : row) start[r + 1]++;
    for (uint64_t i = 0; i < nrow; i++) start[i + 1] += start[i];
    return start;
}
uint64_t sub_row_num(const meta_data_set &m, int s) {
    return m.scalar(GLOBAL_META, "end_row_index", s) - m.scalar(GLOBAL_META, "begin_row_index", s) + 1;
}
}  // namespace

// reorder_val_by_index.cc / reorder_col_by_index.cc: regroup entries in the new row order
void reorder_val_by_index::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &order = m.u(GLOBAL_META, "original_nz_row_indices", s);
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    auto varr = m.get_element(GLOBAL_META, "nz_vals", s)->meta_data_arr;
    uint64_t nrow = sub_row_num(m, s);
    GS_CHECK(nrow == order.size(), "reorder_val_by_index: row count mismatch");
    auto start = old_row_starts(row, nrow);
    std::vector<double> nv(row.size());
    uint64_t p = 0;
    for (uint64_t o : order)
        for (uint64_t k = start[o]; k < start[o + 1]; k++) nv[p++] = varr->read_float_from_arr(k);
    src(GLOBAL_META, "nz_vals");
    replace_f(GLOBAL_META, "nz_vals", std::move(nv), varr->get_data_type());
    is_run = true;
}

void reorder_col_by_index::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &order = m.u(GLOBAL_META, "original_nz_row_indices", s);
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &col = m.u(GLOBAL_META, "nz_col_indices", s);
    uint64_t nrow = sub_row_num(m, s);
    GS_CHECK(nrow == order.size(), "reorder_col_by_index: row count mismatch");
    if (check) {  // reorder_col_by_index.cc:82-93: cols non-decreasing inside a row
        for (uint64_t i = 1; i < row.size(); i++)
            GS_CHECK(row[i] != row[i - 1] || col[i] >= col[i - 1],
                     "reorder_col_by_index: columns not sorted within a row");
    }
    auto start = old_row_starts(row, nrow);
    std::vector<uint64_t> nc(row.size());
    uint64_t p = 0;
    for (uint64_t o : order)
        for (uint64_t k = start[o]; k < start[o + 1]; k++) nc[p++] = col[k];
    src(GLOBAL_META, "nz_col_indices");
    replace_u(GLOBAL_META, "nz_col_indices", std::move(nc));
    is_run = true;
}

// reorder_row_by_index.cc: new row id repeated nnz(old row) times
void reorder_row_by_index::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &order = m.u(GLOBAL_META, "original_nz_row_indices", s);
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t nrow = sub_row_num(m, s);
    GS_CHECK(nrow == order.size(), "reorder_row_by_index: row count mismatch");
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, nrow - 1, 0, row.size() - 1);
    std::vector<uint64_t> nr(row.size());
    uint64_t p = 0;
    for (uint64_t newr = 0; newr < nrow; newr++)
        for (uint64_t k = 0; k < cnt[order[newr]]; k++) nr[p++] = newr;
    src(GLOBAL_META, "nz_row_indices");
    replace_u(GLOBAL_META, "nz_row_indices", std::move(nr));
    is_run = true;
}

// remove_empty_row_in_end_of_sub_matrix.cc:13-70
void remove_empty_row_in_end_of_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", s);
    uint64_t last = m.u(GLOBAL_META, "nz_row_indices", s).back();
    GS_CHECK(last <= e - b, "remove_empty_row: row index beyond sub-matrix");
    if (last < e - b) {
        m.remove_element(GLOBAL_META, "end_row_index", s);
        m.add_scalar(GLOBAL_META, "end_row_index", s, b + last);
        dst(GLOBAL_META, "end_row_index");
    }
    is_run = true;
}

// ----------------------------------------------------------- empty-row padding
// modify_{col,val,row}_*_by_empty_pad_in_submatrix.cc:15-110: a nonzero whose next
// nonzero (the sub-matrix's row count for the last one) lies more than one row further is
// followed by one entry per skipped row -- that row, the nonzero's column, value 0.  The walk
// starts at the first nonzero (leading empty rows stay empty); a nonzero followed by a
// smaller row index is dropped, as the reference's loop emits nothing for it.  The row count
// grows to the largest stored row (:27-33).
namespace {
struct empty_pad_plan {
    std::vector<uint64_t> src, row;  // per output entry: source nonzero, row
    std::vector<uint8_t> pad;        // 1: a padding entry (value 0)
    bool padded = false;
};
empty_pad_plan make_empty_pad(const meta_data_set &m, int s) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    GS_CHECK(!row.empty(), "empty_row_pad: no nonzeros");
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", s);
    if (row.back() > e - b) e = b + row.back();
    const uint64_t rn = e - b + 1;
    empty_pad_plan p;
    p.src.reserve(row.size());
    for (uint64_t i = 0; i < row.size(); i++) {
        const uint64_t r = row[i], nxt = i + 1 == row.size() ? rn : row[i + 1];
        if (nxt == r || nxt == r + 1) {
            p.src.push_back(i); p.row.push_back(r); p.pad.push_back(0);
            continue;
        }
        for (uint64_t id = r; id < nxt; id++) {
            p.src.push_back(i); p.row.push_back(id); p.pad.push_back(id > r);
            if (id > r) p.padded = true;
        }
    }
    return p;
}
}  // namespace

void modify_col_indices_by_empty_pad_in_submatrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_empty_pad(m, target_matrix_id);
    if (p.padded) {
        const auto &col = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
        std::vector<uint64_t> nc(p.src.size());
        for (size_t k = 0; k < nc.size(); k++) nc[k] = col[p.src[k]];
        src(GLOBAL_META, "nz_col_indices");
        replace_u(GLOBAL_META, "nz_col_indices", std::move(nc));
    }
    is_run = true;
}

void modify_vals_by_empty_pad_in_submatrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_empty_pad(m, target_matrix_id);
    if (p.padded) {
        auto va = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
        std::vector<double> nv(p.src.size());
        for (size_t k = 0; k < nv.size(); k++) nv[k] = p.pad[k] ? 0.0 : va->read_float_from_arr(p.src[k]);
        src(GLOBAL_META, "nz_vals");
        replace_f(GLOBAL_META, "nz_vals", std::move(nv), va->get_data_type());
    }
    is_run = true;
}

void modify_row_indices_by_empty_pad_in_submatrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_empty_pad(m, target_matrix_id);
    if (p.padded) {
        src(GLOBAL_META, "nz_row_indices");
        replace_u(GLOBAL_META, "nz_row_indices", std::move(p.row));
    }
    is_run = true;
}

// ------------------------------------------------------------- col pad (A6)
// modify_{col,val,row}_*_by_col_pad_in_sub_matrix.cc: pad each row to a multiple;
// padded entries repeat the row's last column with value 0
namespace {
struct col_pad_plan {
    std::vector<uint64_t> start, cnt, tgt;  // per row (tgt: max-row padding only)
    uint64_t after = 0;
    bool padded = false;
};
col_pad_plan make_col_pad(const meta_data_set &m, int s, int mult, bool check) {
    GS_CHECK(mult >= 2, "col pad multiple must be >= 2 (modify_col_indices_by_col_pad_in_sub_matrix.cc:26)");
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    col_pad_plan p;
    p.cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    p.start.assign(row_num + 1, 0);
    for (uint64_t r = 0; r < row_num; r++) p.start[r + 1] = p.start[r] + p.cnt[r];
    p.after = row.size();
    for (uint64_t r = 0; r < row_num; r++)
        if (p.cnt[r] % mult) p.after += (p.cnt[r] / mult + 1) * mult - p.cnt[r];
    p.padded = p.after != row.size();
    if (check && (double)p.after / (double)row.size() >= padding_bound())
        throw gs_error("col padding rate " + std::to_string((double)p.after / row.size()) +
                       " >= PADDING_RATE_UP_BOUND (modify_col_indices_by_col_pad_in_sub_matrix.cc:103-110)");
    return p;
}
template <class T, class F>
std::vector<T> apply_col_pad(const col_pad_plan &p, int mult, F src_at, T pad_of_last_is_zero_flag) {
    (void)pad_of_last_is_zero_flag;
    std::vector<T> out(p.after);
    uint64_t q = 0;
    for (uint64_t r = 0; r + 1 < p.start.size(); r++) {
        for (uint64_t k = p.start[r]; k < p.start[r + 1]; k++) out[q++] = src_at(k, false);
        if (p.cnt[r] % mult) {
            uint64_t target = (p.cnt[r] / mult + 1) * mult;
            for (uint64_t k = p.cnt[r]; k < target; k++) out[q++] = src_at(p.start[r + 1] - 1, true);
        }
    }
    return out;
}
}  // namespace

void modify_col_indices_by_col_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_col_pad(m, target_matrix_id, multiple_of_each_row_size, check);
    if (p.padded) {
        const auto &col = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
        auto nc = apply_col_pad<uint64_t>(p, multiple_of_each_row_size, [&](uint64_t k, bool) { return col[k]; }, 0);
        src(GLOBAL_META, "nz_col_indices");
        replace_u(GLOBAL_META, "nz_col_indices", std::move(nc));
    }
    is_run = true;
}

void modify_vals_by_col_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_col_pad(m, target_matrix_id, multiple_of_each_row_size, check);
    if (p.padded) {
        auto va = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
        auto nv = apply_col_pad<double>(p, multiple_of_each_row_size,
                                        [&](uint64_t k, bool pad) { return pad ? 0.0 : va->read_float_from_arr(k); }, 0.0);
        src(GLOBAL_META, "nz_vals");
        replace_f(GLOBAL_META, "nz_vals", std::move(nv), va->get_data_type());
    }
    is_run = true;
}

void modify_row_indices_by_col_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_col_pad(m, target_matrix_id, multiple_of_each_row_size, check);
    if (p.padded) {
        const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
        auto nr = apply_col_pad<uint64_t>(p, multiple_of_each_row_size, [&](uint64_t k, bool) { return row[k]; }, 0);
        src(GLOBAL_META, "nz_row_indices");
        replace_u(GLOBAL_META, "nz_row_indices", std::move(nr));
    }
    is_run = true;
}

// ------------------------------------------------------------ row padding
// modify_{col,vals,row}_*_by_row_pad_in_sub_matrix.cc: row_num = end_row_index - begin_row_index
// + 1 (the recorded range, :15-17); when it is not a multiple, one entry per added row is
// appended: column = the last column, value 0, row = row_num + i (:40-47 / :86-107); the
// padding rate is checked against PADDING_RATE_UP_BOUND (:33-38)
namespace {
uint64_t rows_added_by_row_pad(const meta_data_set &m, int s, int mult, bool check) {
    GS_CHECK(mult > 0, "row pad multiple > 0");
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s), e = m.scalar(GLOBAL_META, "end_row_index", s);
    const uint64_t rn = e - b + 1;
    if (rn % (uint64_t)mult == 0) return 0;
    const uint64_t add = (rn / mult + 1) * mult - rn;
    const uint64_t nnz = m.u(GLOBAL_META, "nz_row_indices", s).size();
    GS_CHECK(nnz > 0, "row padding of an empty sub-matrix");
    if (check && (double)(nnz + add) / (double)nnz >= padding_bound())
        throw gs_error("row padding rate >= PADDING_RATE_UP_BOUND (modify_col_indices_by_row_pad_in_sub_matrix.cc:33-38)");
    return add;
}
}  // namespace

void modify_col_indices_by_row_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t add = rows_added_by_row_pad(m, target_matrix_id, multiple, check);
    if (add) {
        std::vector<uint64_t> nc = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
        const uint64_t last = nc.back();
        nc.insert(nc.end(), add, last);
        src(GLOBAL_META, "nz_col_indices");
        replace_u(GLOBAL_META, "nz_col_indices", std::move(nc));
    }
    is_run = true;
}

void modify_vals_by_row_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t add = rows_added_by_row_pad(m, target_matrix_id, multiple, check);
    if (add) {
        auto va = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
        std::vector<double> nv(va->get_len());
        for (uint64_t i = 0; i < nv.size(); i++) nv[i] = va->read_float_from_arr(i);
        nv.insert(nv.end(), add, 0.0);
        src(GLOBAL_META, "nz_vals");
        replace_f(GLOBAL_META, "nz_vals", std::move(nv), va->get_data_type());
    }
    is_run = true;
}

void modify_row_indices_by_row_pad_in_sub_matrix::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t add = rows_added_by_row_pad(m, target_matrix_id, multiple, check);
    if (add) {
        const uint64_t rn = m.scalar(GLOBAL_META, "end_row_index", target_matrix_id) -
                            m.scalar(GLOBAL_META, "begin_row_index", target_matrix_id) + 1;
        std::vector<uint64_t> nr = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
        if (check) GS_CHECK(nr.back() < rn, "row padding: a nonzero past end_row_index (:96-99)");
        for (uint64_t i = 0; i < add; i++) nr.push_back(rn + i);
        src(GLOBAL_META, "nz_row_indices");
        replace_u(GLOBAL_META, "nz_row_indices", std::move(nr));
    }
    is_run = true;
}

// ------------------------------------------- col pad to the parent's max row
// modify_{col,vals,row}_*_by_col_pad_parent_blk_to_max_row_size.cc (padding_with_empty_row
// false): rows [0, row_num) with row_num from the sub-matrix's row range widened to its last
// nonzero's row (:40-52); per parent (GLOBAL: all rows; TBLOCK / WARP: first_row_indices
// ranges) every non-empty row grows to the parent's longest row, pads repeating the row's last
// column with value 0; the padding rate is checked against PADDING_RATE_UP_BOUND (:95-103)
namespace {
col_pad_plan make_max_pad(const meta_data_set &m, int s, POS_TYPE pos, bool with_empty, bool check) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    GS_CHECK(!row.empty(), "max-row padding of an empty sub-matrix");
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", s);
    e = std::max<uint64_t>(e, b + row.back());
    const uint64_t row_num = e - b + 1;
    col_pad_plan p;
    p.cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    p.start.assign(row_num + 1, 0);
    for (uint64_t r = 0; r < row_num; r++) p.start[r + 1] = p.start[r] + p.cnt[r];
    p.tgt = p.cnt;
    std::vector<uint64_t> bounds;
    if (pos == GLOBAL_META) bounds = {0, row_num};
    else bounds = m.u(pos, "first_row_indices", s);
    for (size_t i = 0; i + 1 < bounds.size(); i++) {
        uint64_t mx = 0;
        for (uint64_t r = bounds[i]; r < bounds[i + 1] && r < row_num; r++) mx = std::max(mx, p.cnt[r]);
        for (uint64_t r = bounds[i]; r < bounds[i + 1] && r < row_num; r++)
            if (mx && (p.cnt[r] || with_empty)) {
                p.tgt[r] = mx;
                p.padded = true;  // the reference rewrites the arrays once any row is visited
            }
    }
    p.after = 0;
    for (uint64_t r = 0; r < row_num; r++) p.after += p.tgt[r];
    if (check && (double)p.after / (double)row.size() >= padding_bound())
        throw gs_error("max-row padding rate " + std::to_string((double)p.after / row.size()) +
                       " >= PADDING_RATE_UP_BOUND (modify_col_indices_by_col_pad_parent_blk_to_max_row_size.cc:95-103)");
    return p;
}
// src_at(k, pad, r): a pad repeats element k = the row's last nonzero (an empty row: the last
// nonzero before it, the first one when there is none: :70-72) in row r
template <class T, class F>
std::vector<T> apply_max_pad(const col_pad_plan &p, F src_at) {
    std::vector<T> out;
    out.reserve(p.after);
    for (uint64_t r = 0; r + 1 < p.start.size(); r++) {
        for (uint64_t k = p.start[r]; k < p.start[r + 1]; k++) out.push_back(src_at(k, false, r));
        const uint64_t last = p.start[r + 1] ? p.start[r + 1] - 1 : 0;
        for (uint64_t k = p.cnt[r]; k < p.tgt[r]; k++) out.push_back(src_at(last, true, r));
    }
    return out;
}
}  // namespace

void modify_col_indices_by_col_pad_parent_blk_to_max_row_size::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_max_pad(m, target_matrix_id, parent_pos, padding_with_empty_row, check);
    if (p.padded) {
        const auto &col = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
        auto nc = apply_max_pad<uint64_t>(p, [&](uint64_t k, bool, uint64_t) { return col[k]; });
        src(GLOBAL_META, "nz_col_indices");
        replace_u(GLOBAL_META, "nz_col_indices", std::move(nc));
    }
    is_run = true;
}

void modify_vals_by_col_pad_parent_blk_to_max_row_size::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_max_pad(m, target_matrix_id, parent_pos, padding_with_empty_row, check);
    if (p.padded) {
        auto va = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
        auto nv = apply_max_pad<double>(p, [&](uint64_t k, bool pad, uint64_t) { return pad ? 0.0 : va->read_float_from_arr(k); });
        src(GLOBAL_META, "nz_vals");
        replace_f(GLOBAL_META, "nz_vals", std::move(nv), va->get_data_type());
    }
    is_run = true;
}

void modify_row_indices_by_col_pad_parent_blk_to_max_row_size::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto p = make_max_pad(m, target_matrix_id, parent_pos, padding_with_empty_row, check);
    if (p.padded) {
        const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
        auto nr = apply_max_pad<uint64_t>(p, [&](uint64_t k, bool pad, uint64_t r) { return pad ? r : row[k]; });
        src(GLOBAL_META, "nz_row_indices");
        replace_u(GLOBAL_META, "nz_row_indices", std::move(nr));
    }
    is_run = true;
}

// ------------------------------------------------- fixed row-direction blocks
// get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction.cc:71-97
void get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    GS_CHECK(fixed_row_block_size >= 1, "fixed_row_block_size >= 1");
    if (check) {
        GS_CHECK(m.count_of_metadata_of_diff_pos(TBLOCK_META, s) == 0, "BMT blocking without parent: TBLOCK items exist");
        GS_CHECK(m.count_of_metadata_of_diff_pos(WARP_META, s) == 0, "BMT blocking without parent: WARP items exist");
    }
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    std::vector<uint64_t> fr;
    int in_bmt = 0;
    bool first = true;
    for (uint64_t i = 0; i < row_num; i++) {
        if (first) { fr.push_back(i); first = false; }
        else in_bmt += 1;
        if (in_bmt == fixed_row_block_size) { fr.push_back(i); in_bmt = 0; }
    }
    fr.push_back(row_num);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_row_indices", std::move(fr));
    is_run = true;
}

// get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction.cc:75-100
void get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    std::vector<uint64_t> fn{0};
    int rc = 0;
    uint64_t nz = 0;
    for (uint64_t i = 0; i < row_num; i++) {
        rc += 1;
        nz += cnt[i];
        if (rc == fixed_row_block_size) { fn.push_back(nz); rc = 0; }
    }
    if (rc != fixed_row_block_size && rc != 0) fn.push_back(nz);
    GS_CHECK(fn.back() == row.size(), "first_nz_indices must end at nnz");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_nz_indices", std::move(fn));
    is_run = true;
}

// get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction.cc:136-160: one entry
// (the row index) per chunk of col_size nnz; empty rows get none; no ending
void get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    GS_CHECK(col_size > 0, "col_size > 0");
    GS_CHECK(!m.is_exist(GLOBAL_META, "nz_row_indices_after_interlance_storage", s),
             "col-direction blocking after interleaved storage");
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    std::vector<uint64_t> fr;
    for (uint64_t i = 0; i < row_num; i++) {
        const uint64_t k = (cnt[i] + (uint64_t)col_size - 1) / (uint64_t)col_size;
        for (uint64_t j = 0; j < k; j++) fr.push_back(i);
    }
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_row_indices_without_ending", std::move(fr));
    is_run = true;
}

// get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction.cc:124-150: chunk
// offsets; a row's last chunk holds its remainder
void get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    GS_CHECK(col_size > 0, "col_size > 0");
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    std::vector<uint64_t> fn{0};
    for (uint64_t i = 0; i < row_num; i++)
        for (uint64_t left = cnt[i]; left > 0;) {
            const uint64_t t = std::min<uint64_t>(left, (uint64_t)col_size);
            fn.push_back(fn.back() + t);
            left -= t;
        }
    GS_CHECK(fn.back() == row.size(), "first_nz_indices must end at nnz");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_nz_indices", std::move(fn));
    is_run = true;
}

// ------------------------------------------- col-direction units (A10 and its parents)
namespace {
// the nnz of every row of the sub-matrix (rows up to the real end row)
std::vector<uint64_t> col_row_counts(const meta_data_set &m, int s) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    GS_CHECK(!m.is_exist(GLOBAL_META, "nz_row_indices_after_interlance_storage", s),
             "col-direction blocking after interleaved storage");
    const uint64_t row_num = row_num_of_sub_matrix(m, s);
    return get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
}
// get_begin_rows_of_<unit>_after_fixed_blocking_in_col_direction.cc:75-100: one entry (the
// row) per chunk of c nonzeros of that row; empty rows get none; no ending
std::vector<uint64_t> col_unit_rows(const std::vector<uint64_t> &cnt, uint64_t c) {
    std::vector<uint64_t> fr;
    for (uint64_t i = 0; i < cnt.size(); i++)
        for (uint64_t k = (cnt[i] + c - 1) / c; k; k--) fr.push_back(i);
    return fr;
}
// get_begin_nzs_of_<unit>_after_fixed_blocking_in_col_direction.cc:75-105: chunk starts, a
// row's last chunk holding its remainder, closed by nnz
std::vector<uint64_t> col_unit_nzs(const std::vector<uint64_t> &cnt, uint64_t c) {
    std::vector<uint64_t> fn{0};
    for (uint64_t n : cnt)
        for (uint64_t left = n; left > 0;) {
            const uint64_t t = std::min(left, c);
            fn.push_back(fn.back() + t);
            left -= t;
        }
    return fn;
}
// *_relative_to_{BMTB,BMW}.cc / *_relative_to_parents.cc: the chunks of each row-direction
// parent block, rows minus the parent's first row (rows = true) or nz starts counted from
// the parent's first nonzero (a 0 pushed per parent, the parent's closing offset popped)
std::vector<uint64_t> col_unit_relative(const meta_data_set &m, int s, POS_TYPE parent, uint64_t c, bool rows) {
    const auto cnt = col_row_counts(m, s);
    const auto &pr = m.u(parent, "first_row_indices", s);
    GS_CHECK(pr.size() >= 2 && pr.back() <= cnt.size(), "relative col-direction units need row-direction parents");
    std::vector<uint64_t> out;
    for (size_t p = 0; p + 1 < pr.size(); p++) {
        uint64_t off = 0;
        for (uint64_t r = pr[p]; r < pr[p + 1]; r++)
            for (uint64_t left = cnt[r]; left > 0;) {
                const uint64_t t = std::min(left, c);
                out.push_back(rows ? r - pr[p] : off);
                off += t;
                left -= t;
            }
    }
    return out;
}
}  // namespace

void get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction::run(bool check) {
    GS_CHECK(col_size > 0, "col_size > 0");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_row_indices_without_ending",
              col_unit_rows(col_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)col_size));
    is_run = true;
}
void get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction::run(bool check) {
    GS_CHECK(col_size > 0, "col_size > 0");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_nz_indices", col_unit_nzs(col_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)col_size));
    is_run = true;
}
void get_begin_rows_of_BMTB_after_fixed_blocking_in_col_direction::run(bool check) {
    GS_CHECK(col_size > 0, "col_size > 0");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_row_indices_without_ending",
              col_unit_rows(col_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)col_size));
    is_run = true;
}
void get_begin_nzs_of_BMTB_after_fixed_blocking_in_col_direction::run(bool check) {
    GS_CHECK(col_size > 0, "col_size > 0");
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_nz_indices", col_unit_nzs(col_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)col_size));
    is_run = true;
}
void get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_row_indices");
    replace_u(WARP_META, "first_row_indices_relative_to_BMTB",
              col_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, (uint64_t)col_size, true));
    is_run = true;
}
void get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_row_indices");
    replace_u(WARP_META, "first_nz_indices_relative_to_BMTB",
              col_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, (uint64_t)col_size, false));
    is_run = true;
}
void get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_row_indices");
    replace_u(THREAD_META, "first_row_indices_relative_to_BMTB",
              col_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, (uint64_t)col_size, true));
    is_run = true;
}
void get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMW::run(bool check) {
    src(WARP_META, "first_row_indices");
    replace_u(THREAD_META, "first_row_indices_relative_to_BMW",
              col_unit_relative(*meta_data_set_ptr, target_matrix_id, WARP_META, (uint64_t)col_size, true));
    is_run = true;
}
void get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents::run(bool check) {
    GS_CHECK(parent_pos == TBLOCK_META || parent_pos == WARP_META, "relative BMT nz starts: TBLOCK or WARP parent");
    src(parent_pos, "first_row_indices");
    replace_u(THREAD_META, parent_pos == TBLOCK_META ? "first_nz_indices_relative_to_BMTB" : "first_nz_indices_relative_to_BMW",
              col_unit_relative(*meta_data_set_ptr, target_matrix_id, parent_pos, (uint64_t)col_size, false));
    is_run = true;
}
// remove_item_of_metadata.cc:20-40
void remove_item_of_metadata::run(bool check) {
    auto &m = *meta_data_set_ptr;
    if (check) GS_CHECK(m.is_exist(pos, item_name, target_matrix_id), "remove_item_of_metadata: no item " + item_name);
    src(pos, item_name.c_str());
    m.remove_element(pos, item_name, target_matrix_id);
    is_run = true;
}

namespace {
std::vector<uint64_t> fixed_first_rows(uint64_t row_num, uint64_t rb) {
    std::vector<uint64_t> fr{0};
    uint64_t complete = row_num / rb;
    for (uint64_t i = 0; i < complete; i++) fr.push_back((i + 1) * rb);
    if (row_num % rb) fr.push_back(row_num);
    return fr;
}
std::vector<uint64_t> fixed_first_nzs(const std::vector<uint64_t> &cnt, uint64_t row_num, uint64_t rb) {
    uint64_t nb = row_num / rb + (row_num % rb ? 1 : 0);
    std::vector<uint64_t> fn{0};
    for (uint64_t i = 0; i < nb; i++) {
        uint64_t c = 0;
        for (uint64_t r = i * rb; r < (i + 1) * rb && r < row_num; r++) c += cnt[r];
        fn.push_back(fn.back() + c);
    }
    return fn;
}
}  // namespace

// get_begin_rows_of_BMTBs_after_fixed_blocking_in_row_direction.cc
void get_begin_rows_of_BMTBs_after_fixed_blocking_in_row_direction::run(bool check) {
    GS_CHECK(fixed_row_block_size >= 1, "fixed_row_block_size >= 1");
    uint64_t row_num = row_num_of_sub_matrix(*meta_data_set_ptr, target_matrix_id);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_row_indices", fixed_first_rows(row_num, fixed_row_block_size));
    is_run = true;
}

// get_begin_nzs_of_BMTBs_after_fixed_blocking_in_row_direction.cc
void get_begin_nzs_of_BMTBs_after_fixed_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_nz_indices", fixed_first_nzs(cnt, row_num, fixed_row_block_size));
    is_run = true;
}

void get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB::run(bool check) {
    GS_CHECK(fixed_row_block_size >= 1, "fixed_row_block_size >= 1");
    uint64_t row_num = row_num_of_sub_matrix(*meta_data_set_ptr, target_matrix_id);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_row_indices", fixed_first_rows(row_num, fixed_row_block_size));
    is_run = true;
}

void get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_nz_indices", fixed_first_nzs(cnt, row_num, fixed_row_block_size));
    is_run = true;
}

// get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB.cc
void get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &tr = m.u(TBLOCK_META, "first_row_indices", target_matrix_id);
    std::vector<uint64_t> wr;
    for (uint64_t i = 0; i + 1 < tr.size(); i++)
        for (uint64_t r = tr[i]; r < tr[i + 1]; r += fixed_row_block_size) wr.push_back(r);
    wr.push_back(tr.back());
    src(TBLOCK_META, "first_row_indices");
    replace_u(WARP_META, "first_row_indices", std::move(wr));
    is_run = true;
}

// get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB.cc
void get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &tr = m.u(TBLOCK_META, "first_row_indices", s);
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    std::vector<uint64_t> wn{0};
    for (uint64_t i = 0; i + 1 < tr.size(); i++) {
        for (uint64_t r0 = tr[i]; r0 < tr[i + 1]; r0 += fixed_row_block_size) {
            uint64_t c = 0;
            for (uint64_t r = r0; r < tr[i + 1] && r < r0 + fixed_row_block_size; r++) c += cnt[r];
            wn.push_back(wn.back() + c);
        }
    }
    src(TBLOCK_META, "first_row_indices");
    replace_u(WARP_META, "first_nz_indices", std::move(wn));
    is_run = true;
}

// get_begin_BMWs_of_BMTB_after_blocking_in_row_direction.cc
void get_begin_BMWs_of_BMTB_after_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &tr = m.u(TBLOCK_META, "first_row_indices", s);
    const auto &wr = m.u(WARP_META, "first_row_indices", s);
    std::vector<uint64_t> tb{0};
    uint64_t cur = 0;
    for (uint64_t i = 0; i + 1 < tr.size(); i++) {
        uint64_t num = 0, fr = wr[cur];
        if (check) GS_CHECK(fr == tr[i], "first BMW row != BMTB row");
        while (fr < tr[i + 1]) {
            num++;
            cur++;
            if (cur == wr.size()) break;
            fr = wr[cur];
        }
        tb.push_back(tb.back() + num);
    }
    src(WARP_META, "first_row_indices");
    replace_u(TBLOCK_META, "first_BMW_indices", std::move(tb));
    is_run = true;
}

// ------------------------------------------------------ nnz-direction (A9)
// modify_*_by_nnz_pad.cc:14-75
namespace {
uint64_t nnz_pad_target(uint64_t nnz, int t, bool check) {
    if (nnz % t == 0) return nnz;
    uint64_t nn = (nnz / t + 1) * t;
    if (check && (double)nn / (double)nnz >= padding_bound())
        throw gs_error("nnz padding rate " + std::to_string((double)nn / nnz) +
                       " >= PADDING_RATE_UP_BOUND (modify_col_indices_by_nnz_pad.cc)");
    return nn;
}
}  // namespace

void modify_col_indices_by_nnz_pad::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto c = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
    uint64_t nn = nnz_pad_target(c.size(), nnz_target, check);
    if (nn != c.size()) {
        c.resize(nn, c.back());
        src(GLOBAL_META, "nz_col_indices");
        replace_u(GLOBAL_META, "nz_col_indices", std::move(c));
    }
    is_run = true;
}

void modify_vals_by_nnz_pad::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto va = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
    uint64_t nn = nnz_pad_target(va->get_len(), nnz_target, check);
    if (nn != va->get_len()) {
        std::vector<double> v = va->f();
        v.resize(nn, 0.0);
        src(GLOBAL_META, "nz_vals");
        replace_f(GLOBAL_META, "nz_vals", std::move(v), va->get_data_type());
    }
    is_run = true;
}

void modify_row_indices_by_nnz_pad::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto r = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t nn = nnz_pad_target(r.size(), nnz_target, check);
    if (nn != r.size()) {
        r.resize(nn, r.back());
        src(GLOBAL_META, "nz_row_indices");
        replace_u(GLOBAL_META, "nz_row_indices", std::move(r));
    }
    is_run = true;
}

// get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction.cc
void get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    std::vector<uint64_t> fr;
    for (uint64_t i = 0; i < row.size(); i += nnz_per_BMT) fr.push_back(row[i]);
    GS_CHECK(row_num > fr.back(), "BMT first row beyond row count");
    fr.push_back(row_num);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_row_indices", std::move(fr));
    is_run = true;
}

// get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction.cc
void get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    uint64_t nnz = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id).size();
    std::vector<uint64_t> fn;
    for (uint64_t i = 0; i < nnz; i += nnz_per_BMT) fn.push_back(i);
    fn.push_back(nnz);
    src(GLOBAL_META, "nz_row_indices");
    replace_u(THREAD_META, "first_nz_indices", std::move(fn));
    is_run = true;
}

// get_BMT_size_of_each_parent.cc: one size per parent block, or no item at all when
// the BMT sizes inside a parent differ (:118-121)
void get_BMT_size_of_each_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &fn = m.u(THREAD_META, "first_nz_indices", s);
    std::vector<uint64_t> sizes;
    if (parent_pos == GLOBAL_META) {
        uint64_t sz = fn.size() >= 2 ? fn[1] - fn[0] : 0;
        for (uint64_t i = 0; i + 1 < fn.size(); i++)
            if (fn[i + 1] - fn[i] != sz) { is_run = true; return; }
        sizes.push_back(sz);
    } else {
        const auto &pn = m.u(parent_pos, "first_nz_indices", s);
        const std::vector<uint64_t> *pb = row_direction_blocking ? &m.u(parent_pos, "first_BMT_indices", s) : nullptr;
        uint64_t cur = 0;
        for (uint64_t p = 0; p + 1 < pn.size(); p++) {
            uint64_t sz = 0;
            bool seen = false;
            uint64_t cur_nz = fn[cur];
            while (cur_nz < pn[p + 1]) {
                uint64_t b = fn[cur + 1] - fn[cur];
                if (!seen) { sz = b; seen = true; }
                else if (b != sz) { is_run = true; return; }
                cur++;
                cur_nz = fn[cur];
            }
            if (row_direction_blocking && pn[p] == pn[p + 1])
                while (cur < (*pb)[p + 1]) cur++;
            sizes.push_back(sz);
        }
    }
    src(THREAD_META, "first_nz_indices");
    replace_u(parent_pos, "BMT_size_of_each_blk", std::move(sizes));
    is_run = true;
}

// ------------------------------------------- nnz-direction WARP / TBLOCK units
namespace {
// get_begin_rows_of_{BMW,BMTB}_after_fixed_blocking_in_nnz_direction.cc:20-40
std::vector<uint64_t> nnz_unit_rows(const meta_data_set &m, int s, uint64_t k) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", s);
    if (e < b + row.back()) e = b + row.back();
    std::vector<uint64_t> fr;
    for (uint64_t i = 0; i < row.size(); i += k) fr.push_back(row[i]);
    fr.push_back(e - b + 1);
    return fr;
}
// get_begin_nzs_of_{BMW,BMTB}_after_fixed_blocking_in_nnz_direction.cc:18-30
std::vector<uint64_t> nnz_unit_nzs(uint64_t nnz, uint64_t k) {
    std::vector<uint64_t> fn;
    for (uint64_t i = 0; i < nnz; i += k) fn.push_back(i);
    fn.push_back(nnz);
    return fn;
}
// *_relative_to_{BMTB,BMW}.cc:25-45: the parent advances by one when a unit start reaches
// the next parent's first nonzero (an `if`, as in the reference: parents are never skipped
// when their sizes are multiples of the unit size, which the operators require)
std::vector<uint64_t> nnz_unit_relative(const meta_data_set &m, int s, POS_TYPE parent, uint64_t k, bool rows) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &pn = m.u(parent, "first_nz_indices", s);
    const std::vector<uint64_t> *pr = rows ? &m.u(parent, "first_row_indices", s) : nullptr;
    std::vector<uint64_t> out;
    uint64_t pid = 0;
    for (uint64_t i = 0; i < row.size(); i += k) {
        GS_CHECK(pid + 1 < pn.size(), "nnz-direction unit beyond its parents");
        if (i >= pn[pid + 1]) pid++;
        out.push_back(rows ? row[i] - (*pr)[pid] : i - pn[pid]);
    }
    return out;
}
// children per parent: the first child index of every parent, parents start on a child
std::vector<uint64_t> children_of_parents(const std::vector<uint64_t> &cn, const std::vector<uint64_t> &pn,
                                          const char *what) {
    std::vector<uint64_t> out{0};
    uint64_t cur = 0;
    for (uint64_t p = 0; p + 1 < pn.size(); p++) {
        GS_CHECK(cur < cn.size() && cn[cur] == pn[p], std::string(what) + ": a parent does not start on a child");
        uint64_t num = 0;
        while (cn[cur] < pn[p + 1]) {
            num++;
            cur++;
            GS_CHECK(cur < cn.size(), std::string(what) + ": children end before the parents");
        }
        out.push_back(out.back() + num);
    }
    return out;
}
// one size per parent when all children of it have the same number of nonzeros; a
// parent with mixed sizes: nullopt (get_BMW_size_of_each_parent.cc returns without
// writing the array)
bool equal_sizes(const std::vector<uint64_t> &cn, const std::vector<uint64_t> *pn, std::vector<uint64_t> &out) {
    out.clear();
    if (!pn) {
        uint64_t sz = 0;
        for (uint64_t i = 0; i + 1 < cn.size(); i++) {
            const uint64_t b = cn[i + 1] - cn[i];
            if (i == 0) sz = b;
            else if (b != sz) return false;
        }
        out.push_back(sz);
        return true;
    }
    uint64_t cur = 0;
    for (uint64_t p = 0; p + 1 < pn->size(); p++) {
        uint64_t sz = 0;
        bool seen = false;
        while (cur + 1 < cn.size() && cn[cur] < (*pn)[p + 1]) {
            const uint64_t b = cn[cur + 1] - cn[cur];
            if (!seen) { sz = b; seen = true; }
            else if (b != sz) return false;
            cur++;
        }
        out.push_back(sz);
    }
    return true;
}
}  // namespace

void get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction::run(bool check) {
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_row_indices", nnz_unit_rows(*meta_data_set_ptr, target_matrix_id, nnz_per_BMW));
    is_run = true;
}
void get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction::run(bool check) {
    src(GLOBAL_META, "nz_row_indices");
    replace_u(WARP_META, "first_nz_indices",
              nnz_unit_nzs(meta_data_set_ptr->u(GLOBAL_META, "nz_row_indices", target_matrix_id).size(), nnz_per_BMW));
    is_run = true;
}
void get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_row_indices");
    replace_u(WARP_META, "first_row_indices_relative_to_BMTB",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, nnz_per_BMW, true));
    is_run = true;
}
void get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_nz_indices");
    replace_u(WARP_META, "first_nz_indices_relative_to_BMTB",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, nnz_per_BMW, false));
    is_run = true;
}
void get_begin_rows_of_BMTB_after_fixed_blocking_in_nnz_direction::run(bool check) {
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_row_indices", nnz_unit_rows(*meta_data_set_ptr, target_matrix_id, nnz_per_BMTB));
    is_run = true;
}
void get_begin_nzs_of_BMTB_after_fixed_blocking_in_nnz_direction::run(bool check) {
    src(GLOBAL_META, "nz_row_indices");
    replace_u(TBLOCK_META, "first_nz_indices",
              nnz_unit_nzs(meta_data_set_ptr->u(GLOBAL_META, "nz_row_indices", target_matrix_id).size(), nnz_per_BMTB));
    is_run = true;
}
void get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_row_indices");
    replace_u(THREAD_META, "first_row_indices_relative_to_BMTB",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, nnz_per_BMT, true));
    is_run = true;
}
void get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB::run(bool check) {
    src(TBLOCK_META, "first_nz_indices");
    replace_u(THREAD_META, "first_nz_indices_relative_to_BMTB",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, TBLOCK_META, nnz_per_BMT, false));
    is_run = true;
}
void get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW::run(bool check) {
    src(WARP_META, "first_row_indices");
    replace_u(THREAD_META, "first_row_indices_relative_to_BMW",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, WARP_META, nnz_per_BMT, true));
    is_run = true;
}
void get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW::run(bool check) {
    src(WARP_META, "first_nz_indices");
    replace_u(THREAD_META, "first_nz_indices_relative_to_BMW",
              nnz_unit_relative(*meta_data_set_ptr, target_matrix_id, WARP_META, nnz_per_BMT, false));
    is_run = true;
}
// get_begin_BMWs_of_BMTB_after_blocking.cc:20-60
void get_begin_BMWs_of_BMTB_after_blocking::run(bool check) {
    auto &m = *meta_data_set_ptr;
    src(WARP_META, "first_nz_indices");
    src(TBLOCK_META, "first_nz_indices");
    replace_u(TBLOCK_META, "first_BMW_indices",
              children_of_parents(m.u(WARP_META, "first_nz_indices", target_matrix_id),
                                  m.u(TBLOCK_META, "first_nz_indices", target_matrix_id), "get_begin_BMWs_of_BMTB_after_blocking"));
    is_run = true;
}
// get_begin_BMTs_of_specific_parent_after_blocking.cc:20-75
void get_begin_BMTs_of_specific_parent_after_blocking::run(bool check) {
    auto &m = *meta_data_set_ptr;
    GS_CHECK(parent_pos == TBLOCK_META || parent_pos == WARP_META, "BMT parent must be TBLOCK or WARP");
    src(THREAD_META, "first_nz_indices");
    src(parent_pos, "first_nz_indices");
    replace_u(parent_pos, "first_BMT_indices",
              children_of_parents(m.u(THREAD_META, "first_nz_indices", target_matrix_id),
                                  m.u(parent_pos, "first_nz_indices", target_matrix_id),
                                  "get_begin_BMTs_of_specific_parent_after_blocking"));
    is_run = true;
}
// get_BMW_size_of_each_parent.cc:20-150 (mixed sizes: nothing written)
void get_BMW_size_of_each_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    std::vector<uint64_t> sizes;
    const std::vector<uint64_t> *pn = parent_pos == GLOBAL_META ? nullptr : &m.u(parent_pos, "first_nz_indices", target_matrix_id);
    if (equal_sizes(m.u(WARP_META, "first_nz_indices", target_matrix_id), pn, sizes)) {
        src(WARP_META, "first_nz_indices");
        replace_u(parent_pos, "BMW_size_of_each_blk", std::move(sizes));
    }
    is_run = true;
}
// get_BMTB_size.cc:20-95 (mixed sizes assert)
void get_BMTB_size::run(bool check) {
    auto &m = *meta_data_set_ptr;
    std::vector<uint64_t> sizes;
    GS_CHECK(equal_sizes(m.u(TBLOCK_META, "first_nz_indices", target_matrix_id), nullptr, sizes),
             "get_BMTB_size: the BMTB sizes are not the same (get_BMTB_size.cc:81-85)");
    src(TBLOCK_META, "first_nz_indices");
    replace_u(GLOBAL_META, "BMTB_size_of_each_blk", std::move(sizes));
    is_run = true;
}

// ------------------------------------------------------------ bitmaps
// thread_bit_map.cc:14-92.  Bit i of map b is 1 iff nz first_nz[b]+i starts a row
// (LSB = first nz).  With a parent level, the head of every parent_size-th BMT is
// forced to 1.  The reference's division by zero (no GLOBAL BMT_size_of_each_blk)
// becomes an error; its one-past-the-end write never reaches an output.
void thread_bit_map::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &fn = m.u(THREAD_META, "first_nz_indices", s);
    GS_CHECK(fn.back() == row.size(), "thread_bit_map: first_nz_indices must end at nnz (thread_bit_map.cc:43)");
    uint64_t nnz = row.size(), nb = fn.size() - 1;
    std::vector<uint8_t> bit(nnz);
    bit[0] = 1;
    for (uint64_t j = 1; j < nnz; j++) bit[j] = row[j] != row[j - 1];
    if (parent_flag) {
        GS_CHECK(m.is_exist(GLOBAL_META, "BMT_size_of_each_blk", s),
                 "thread_bit_map: GLOBAL BMT_size_of_each_blk missing (reference divides by zero, thread_bit_map.cc:56)");
        uint64_t ts = fn[1] - fn[0];
        for (uint64_t i = 0; i < nnz / ts + 1; i += (uint64_t)parent_size)
            if (i * ts < nnz) bit[i * ts] = 1;
    }
    std::vector<uint64_t> maps(nb);
    for (uint64_t i = 0; i < nb; i++) {
        uint64_t mm = 0;
        for (uint64_t j = fn[i + 1]; j-- > fn[i];) mm = (mm << 1) | bit[j];
        maps[i] = mm;
    }
    src(GLOBAL_META, "nz_row_indices");
    src(THREAD_META, "first_nz_indices");
    replace_u(THREAD_META, "thread_bit_map", std::move(maps));
    is_run = true;
}

// segment_empty_flag.cc:14-75
void segment_empty_flag::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &fn = m.u(THREAD_META, "first_nz_indices", s);
    uint64_t nb = fn.size() - 1;
    std::vector<uint8_t> flag(nb, 0);
    for (uint64_t j = 0; j < nb; j++)
        for (uint64_t i = fn[j] + 1; i < fn[j + 1]; i++)
            if (row[i] - row[i - 1] > 1) { flag[j] = 1; break; }
    std::vector<uint64_t> out;
    for (uint64_t i = 0; i < nb; i += (uint64_t)size) {
        uint64_t k = std::min<uint64_t>(i + size - 1, nb - 1), cur = 0;
        for (uint64_t j = k + 1; j-- > i;) cur = (cur << 1) | flag[j];
        out.push_back(cur);
    }
    replace_u(THREAD_META, "segment_empty_flag", std::move(out));
    is_run = true;
}

// segment_empty_row_indices.cc
void segment_empty_row_indices::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &fn = m.u(THREAD_META, "first_nz_indices", s);
    std::vector<uint64_t> out;
    for (uint64_t j = 0; j + 1 < fn.size(); j++) {
        uint64_t r0 = row[fn[j]];
        out.push_back(0);
        for (uint64_t i = fn[j] + 1; i < fn[j + 1]; i++)
            if (row[i] != row[i - 1]) out.push_back(row[i] - r0);
    }
    replace_u(THREAD_META, "segment_empty_row_indices", std::move(out));
    is_run = true;
}

// segment_offset.cc: the count pending after the last non-empty map is not written
void segment_offset::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const char *src_name = m.is_exist(THREAD_META, "thread_bit_map", s) ? "thread_bit_map" : "bit_map_of_thread";
    const auto &bm = m.u(THREAD_META, src_name, s);
    std::vector<uint64_t> out(bm.size(), 0);
    uint64_t count = 0, prev = 0;
    for (uint64_t j = 1; j < bm.size(); j++) {
        if (bm[j] == 0 && ((j % size != 0) || !parent_flag)) count++;
        else { out[prev] = count; count = 0; prev = j; }
    }
    replace_u(THREAD_META, "segment_offset", std::move(out));
    is_run = true;
}

// segment_ptr.cc: exclusive running count of row segments per BMT
void segment_ptr::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const auto &fn = m.u(THREAD_META, "first_nz_indices", s);
    std::vector<uint64_t> out{0};
    uint64_t c = 0;
    for (uint64_t j = 0; j + 2 < fn.size(); j++) {
        c += 1;
        for (uint64_t i = fn[j] + 1; i < fn[j + 1]; i++)
            if (row[i] != row[i - 1]) c += 1;
        out.push_back(c);
    }
    replace_u(THREAD_META, "segment_ptr", std::move(out));
    is_run = true;
}

// get_begin_{rows,nzs,BMTs}_after_merge_thread.cc
static std::vector<uint64_t> merge_every(const std::vector<uint64_t> &a, int k) {
    std::vector<uint64_t> out;
    for (uint64_t j = 0; j + 1 < a.size(); j += (uint64_t)k) out.push_back(a[j]);
    out.push_back(a.back());
    return out;
}
void get_begin_rows_after_merge_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const char *n = m.is_exist(THREAD_META, "first_row_indices", target_matrix_id) ? "first_row_indices"
                                                                                   : "first_row_indices_without_ending";
    replace_u(pos, "first_row_indices", merge_every(m.u(THREAD_META, n, target_matrix_id), merge_num));
    is_run = true;
}
void get_begin_nzs_after_merge_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    replace_u(pos, "first_nz_indices", merge_every(m.u(THREAD_META, "first_nz_indices", target_matrix_id), merge_num));
    is_run = true;
}
void get_begin_BMTs_after_merge_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    uint64_t n = m.u(THREAD_META, "first_nz_indices", target_matrix_id).size();
    std::vector<uint64_t> out;
    for (uint64_t j = 0; j + 1 < n; j += (uint64_t)merge_num) out.push_back(j);
    out.push_back(n - 1);
    replace_u(pos, "first_BMT_indices", std::move(out));
    is_run = true;
}

// get_begin_{rows,nzs}_relative_to_parent_after_merge_thread.cc: offsets of each BMT
// from the first BMT of its merged parent; the loop stops one short of the array
// end, so over the ending-less row array the last BMT gets no entry (reference
// behaviour).  Rows go to <pos>_..., nz offsets to THREAD_... (as the reference).
static std::vector<uint64_t> relative_to_merged(const std::vector<uint64_t> &a, int k) {
    std::vector<uint64_t> out;
    for (uint64_t j = 0; j + 1 < a.size(); j += (uint64_t)k)
        for (uint64_t i = j; i < j + (uint64_t)k && i + 1 < a.size(); i++) out.push_back(a[i] - a[j]);
    return out;
}
static const char *relative_name(POS_TYPE pos, bool row) {
    GS_CHECK(pos == WARP_META || pos == TBLOCK_META, "relative indices need a WARP or TBLOCK parent");
    if (row)
        return pos == WARP_META ? "first_row_indices_relative_to_BMW" : "first_row_indices_relative_to_BMTB";
    return pos == WARP_META ? "first_nz_indices_relative_to_BMW" : "first_nz_indices_relative_to_BMTB";
}
void get_begin_rows_relative_to_parent_after_merge_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const char *n = m.is_exist(THREAD_META, "first_row_indices", target_matrix_id) ? "first_row_indices"
                                                                                   : "first_row_indices_without_ending";
    replace_u(pos, relative_name(pos, true), relative_to_merged(m.u(THREAD_META, n, target_matrix_id), merge_num));
    is_run = true;
}
void get_begin_nzs_relative_to_parent_after_merge_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    replace_u(THREAD_META, relative_name(pos, false),
              relative_to_merged(m.u(THREAD_META, "first_nz_indices", target_matrix_id), merge_num));
    is_run = true;
}

// parent_bit_map_of_thread.cc: a BMT's bit is set when it starts a new row or a
// new parent.  WARP: one word per VECTOR_WIDTH BMTs, bit t = BMT i+t (bits past
// 64 shift out of the unsigned long, as in the reference).  TBLOCK: one 0/1 entry
// per BMT under THREAD_META; the parent head at first_BMT_indices' ending (= the
// BMT count) would be written one past the end in the reference and is skipped.
void parent_bit_map_of_thread::run(bool check) {
    auto &m = *meta_data_set_ptr;
    int s = target_matrix_id;
    const auto &fr = m.u(THREAD_META, "first_row_indices_without_ending", s);
    const uint64_t n = fr.size();
    std::vector<uint8_t> bit(n, 0);
    if (n) bit[0] = 1;
    for (uint64_t j = 1; j < n; j++) bit[j] = fr[j] != fr[j - 1];
    std::vector<uint64_t> out;
    if (pos == WARP_META) {
        const uint64_t vw = (uint64_t)get_config().VECTOR_WIDTH;
        GS_CHECK(vw >= 1, "VECTOR_WIDTH >= 1");
        for (uint64_t i = 0; i < n; i += vw) bit[i] = 1;
        for (uint64_t i = 0; i < n; i += vw) {
            const uint64_t k = std::min(i + vw - 1, n - 1);
            uint64_t map = 0;
            for (uint64_t j = k + 1; j-- > i;) map = (map << 1) | bit[j];
            out.push_back(map);
        }
        replace_u(WARP_META, "bit_map_of_thread", std::move(out));
    } else {
        GS_CHECK(pos == TBLOCK_META, "parent_bit_map_of_thread: parent must be WARP or TBLOCK");
        for (uint64_t b : m.u(TBLOCK_META, "first_BMT_indices", s))
            if (b < n) bit[b] = 1;
        out.assign(bit.begin(), bit.end());
        replace_u(THREAD_META, "bit_map_of_thread", std::move(out));
    }
    src(THREAD_META, "first_row_indices_without_ending");
    is_run = true;
}

// ---------------------------------------------------------- balanced (A11)
// data_transform_common.cc:934-957 (`unsigned int` counters kept)
std::vector<uint64_t> get_begin_nzs_of_child_after_balance_blocking_in_row_direction(
    const std::vector<uint64_t> &cnt, uint64_t per) {
    std::vector<uint64_t> out{0};
    uint32_t c = 0, tot = 0;
    for (uint64_t x : cnt) {
        c += (uint32_t)x;
        tot += (uint32_t)x;
        if (c >= per) { out.push_back(tot); c = 0; }
    }
    if (c != 0) out.push_back(tot);
    return out;
}
// data_transform_common.cc:960-989
std::vector<uint64_t> get_begin_rows_of_child_after_balance_blocking_in_row_direction(
    const std::vector<uint64_t> &cnt, uint64_t per, uint64_t row_num) {
    std::vector<uint64_t> out{0};
    uint64_t c = 0;
    for (uint64_t i = 0; i < row_num; i++) {
        c += cnt[i];
        if (c >= per) { out.push_back(i + 1); c = 0; }
    }
    if (out.back() < row_num) {
        GS_CHECK(c != 0, "balanced blocking: empty rows after the last cut (data_transform_common.cc:984)");
        out.push_back(row_num);
    }
    return out;
}

void get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    replace_u(WARP_META, "first_row_indices",
              get_begin_rows_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval, row_num));
    is_run = true;
}

// balanced BMWs inside BMTBs (data_transform_common.cc:794-901): per BMTB a new BMW after the
// row whose running count reaches nnz_per_interval, never at the BMTB's last row (the next
// BMTB starts one anyway); absolute arrays end with row_num / the last BMTB nz, the
// relative ones restart at 0 per BMTB and have no ending.  row_num widens the recorded range to
// the last nonzero's row (get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB.cc:33-40)
namespace {
struct bmw_in_bmtb {
    std::vector<uint64_t> rows, rows_rel, nzs, nzs_rel;
};
bmw_in_bmtb balanced_in_parent(const meta_data_set &m, int s, POS_TYPE parent, uint64_t per) {
    GS_CHECK(per > 0, "nnz_per_interval > 0");
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    GS_CHECK(!row.empty(), "balanced BMWs of an empty sub-matrix");
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s);
    const uint64_t e = std::max<uint64_t>(m.scalar(GLOBAL_META, "end_row_index", s), b + row.back());
    const uint64_t row_num = e - b + 1;
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    const auto &pr = m.u(parent, "first_row_indices", s);
    const auto &pn = m.u(parent, "first_nz_indices", s);
    GS_CHECK(pr.size() == pn.size() && pr.size() >= 2, "parent first_row_indices / first_nz_indices disagree");
    bmw_in_bmtb o;
    for (size_t j = 0; j + 1 < pr.size(); j++) {
        o.rows.push_back(pr[j]);
        o.rows_rel.push_back(0);
        o.nzs.push_back(pn[j]);
        o.nzs_rel.push_back(0);
        uint64_t run = 0, in_blk = 0;
        for (uint64_t i = pr[j]; i < pr[j + 1]; i++) {
            run += cnt[i];
            in_blk += cnt[i];
            if (run >= per && i != pr[j + 1] - 1) {
                o.rows.push_back(i + 1);
                o.rows_rel.push_back(i + 1 - pr[j]);
                o.nzs.push_back(pn[j] + in_blk);
                o.nzs_rel.push_back(in_blk);
                run = 0;
            }
        }
    }
    o.rows.push_back(row_num);
    o.nzs.push_back(pn.back());
    return o;
}
bmw_in_bmtb balanced_bmw_in_bmtb(const meta_data_set &m, int s, uint64_t per) { return balanced_in_parent(m, s, TBLOCK_META, per); }
std::string rel_name(const char *base, POS_TYPE parent) {
    return std::string(base) + (parent == WARP_META ? "_relative_to_BMW" : "_relative_to_BMTB");
}
}  // namespace

void get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_in_parent::run(bool check) {
    replace_u(THREAD_META, "first_row_indices", balanced_in_parent(*meta_data_set_ptr, target_matrix_id, parent_pos, nnz_per_interval).rows);
    is_run = true;
}
void get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent::run(bool check) {
    replace_u(THREAD_META, rel_name("first_row_indices", parent_pos).c_str(),
              balanced_in_parent(*meta_data_set_ptr, target_matrix_id, parent_pos, nnz_per_interval).rows_rel);
    is_run = true;
}
void get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_in_parent::run(bool check) {
    replace_u(THREAD_META, "first_nz_indices", balanced_in_parent(*meta_data_set_ptr, target_matrix_id, parent_pos, nnz_per_interval).nzs);
    is_run = true;
}
void get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent::run(bool check) {
    replace_u(THREAD_META, rel_name("first_nz_indices", parent_pos).c_str(),
              balanced_in_parent(*meta_data_set_ptr, target_matrix_id, parent_pos, nnz_per_interval).nzs_rel);
    is_run = true;
}

void get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB::run(bool check) {
    replace_u(WARP_META, "first_row_indices", balanced_bmw_in_bmtb(*meta_data_set_ptr, target_matrix_id, nnz_per_interval).rows);
    is_run = true;
}
void get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB::run(bool check) {
    replace_u(WARP_META, "first_row_indices_relative_to_BMTB",
              balanced_bmw_in_bmtb(*meta_data_set_ptr, target_matrix_id, nnz_per_interval).rows_rel);
    is_run = true;
}
void get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB::run(bool check) {
    replace_u(WARP_META, "first_nz_indices", balanced_bmw_in_bmtb(*meta_data_set_ptr, target_matrix_id, nnz_per_interval).nzs);
    is_run = true;
}
void get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB::run(bool check) {
    replace_u(WARP_META, "first_nz_indices_relative_to_BMTB",
              balanced_bmw_in_bmtb(*meta_data_set_ptr, target_matrix_id, nnz_per_interval).nzs_rel);
    is_run = true;
}

void get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    replace_u(WARP_META, "first_nz_indices",
              get_begin_nzs_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval));
    is_run = true;
}

// balanced TBLOCK level (get_begin_rows_of_BMTB_after_nnz_blocking_in_row_direction.cc:65-86,
// get_begin_nzs_of_BMTB_after_nnz_blocking_in_row_direction.cc:55-80): same split rules, TBLOCK arrays
void get_begin_rows_of_BMTB_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    auto v = get_begin_rows_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval, row_num);
    if (check) GS_CHECK(v.back() == row_num, "balanced BMTB rows must end at the row count (:77)");
    replace_u(TBLOCK_META, "first_row_indices", std::move(v));
    src(GLOBAL_META, "nz_row_indices");
    is_run = true;
}

void get_begin_nzs_of_BMTB_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    auto v = get_begin_nzs_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval);
    if (check) GS_CHECK(v.back() == row.size(), "balanced BMTB nzs must end at nnz (:72-75)");
    replace_u(TBLOCK_META, "first_nz_indices", std::move(v));
    src(GLOBAL_META, "nz_row_indices");
    is_run = true;
}

// balanced THREAD level, no parent (get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction.cc:60-81,
// get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction.cc:53-88)
void get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    replace_u(THREAD_META, "first_row_indices",
              get_begin_rows_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval, row_num));
    src(GLOBAL_META, "nz_row_indices");
    is_run = true;
}

void get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    auto v = get_begin_nzs_of_child_after_balance_blocking_in_row_direction(cnt, nnz_per_interval);
    if (check) GS_CHECK(v.back() == row.size(), "balanced BMT nzs must end at nnz (:78-81)");
    replace_u(THREAD_META, "first_nz_indices", std::move(v));
    src(GLOBAL_META, "nz_row_indices");
    is_run = true;
}

// ------------------------------------------------------- merge path (A11)
// get_begin_rows_of_level_after_merge_path.cc:58-94 and
// get_begin_nzs_of_level_after_merge_path.cc:60-95.  The reference finds, for
// every level start i = 0, ws, 2ws, ... < count, the first non-empty row j with
// total_path[j] > i by a linear scan from j = 0 (quadratic); i grows, so the
// scan resumes where the previous one stopped (same j, same outputs).
// total_path[j] = sum_{t<=j} (nnz_t + 1) - 1 over non-empty rows; the level
// records row = that row's index and nz = i - j; the nz list ends with nnz.
void merge_path_levels(const std::vector<uint64_t> &cnt, uint64_t ws, std::vector<uint64_t> *level_rows,
                       std::vector<uint64_t> *level_nzs) {
    GS_CHECK(ws > 0, "work_size > 0");
    std::vector<uint64_t> total_path, path_row;
    uint64_t count = 0, nnz = 0;
    bool first = true;
    for (uint64_t i = 0; i < cnt.size(); i++) {
        nnz += cnt[i];
        if (cnt[i] != 0) {
            count += 1;
            if (first) { first = false; count -= 1; }
            count += cnt[i];
            total_path.push_back(count);
            path_row.push_back(i);
        }
    }
    uint64_t j = 0;
    for (uint64_t i = 0; i < count; i += ws) {
        while (j < total_path.size() && total_path[j] <= i) j++;
        if (j == total_path.size()) break;  // unreachable: total_path.back() == count > i
        if (level_rows) level_rows->push_back(path_row[j]);
        if (level_nzs) level_nzs->push_back(i - j);
    }
    if (level_nzs) level_nzs->push_back(nnz);
}

static std::vector<uint64_t> merge_path_row_counts(const meta_data_set &m, int s) {
    // :26-50 of either file: row_num from begin/end_row_index raised to the last row in the data
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    uint64_t row_num = row_num_of_sub_matrix(m, s);
    return get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
}

void get_begin_rows_of_level_after_merge_path::run(bool check) {
    GS_CHECK(work_size > 0, "work_size > 0");
    std::vector<uint64_t> rows;
    merge_path_levels(merge_path_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)work_size, &rows, nullptr);
    GS_CHECK(!rows.empty(), "merge path over a sub-matrix without nonzeros");
    replace_u(pos, "first_row_indices_without_ending", std::move(rows));
    src(GLOBAL_META, "nz_row_indices");
    src(GLOBAL_META, "begin_row_index");
    src(GLOBAL_META, "end_row_index");
    is_run = true;
}

void get_begin_nzs_of_level_after_merge_path::run(bool check) {
    GS_CHECK(work_size > 0, "work_size > 0");
    std::vector<uint64_t> nzs;
    merge_path_levels(merge_path_row_counts(*meta_data_set_ptr, target_matrix_id), (uint64_t)work_size, nullptr, &nzs);
    replace_u(pos, "first_nz_indices", std::move(nzs));
    src(GLOBAL_META, "nz_row_indices");
    src(GLOBAL_META, "begin_row_index");
    src(GLOBAL_META, "end_row_index");
    is_run = true;
}

// ----------------------------------------------- interleaved storage (§8f rank 2)
// modify_col_indices_by_interlance_storage.cc:45-116 (the vals / rows files are the same
// loop): GLOBAL parent -> one block of BMT_num = nnz / size BMTs, spacing BMT_num;
// TBLOCK / WARP parent -> per parent p, BMTs [first_BMT[p], first_BMT[p+1]) of size
// BMT_size_of_each_blk[p], spacing = their count, offset = the nonzeros before p
std::vector<uint64_t> interlance_storage_permutation(const meta_data_set &m, POS_TYPE parent_pos, int s, bool check) {
    const uint64_t n = m.u(GLOBAL_META, "nz_col_indices", s).size();
    const auto &bsz = m.u(parent_pos, "BMT_size_of_each_blk", s);
    std::vector<uint64_t> to(n);
    if (parent_pos == GLOBAL_META) {
        GS_CHECK(!bsz.empty() && bsz[0] > 0, "interleaved storage: BMT_size_of_each_blk missing");
        const uint64_t sz = bsz[0];
        if (check) GS_CHECK(n % sz == 0, "interleaved storage: nnz is not a multiple of the BMT size (:57)");
        const uint64_t nb = n / sz;
        for (uint64_t b = 0; b < nb; b++)
            for (uint64_t i = 0; i < sz; i++) to[i + b * sz] = b + i * nb;
    } else {
        const auto &fb = m.u(parent_pos, "first_BMT_indices", s);
        uint64_t base = 0;
        for (uint64_t p = 0; p + 1 < fb.size(); p++) {
            const uint64_t nb = fb[p + 1] - fb[p], sz = bsz[p];
            if (check) GS_CHECK(m.u(parent_pos, "first_nz_indices", s)[p] == base, "interleaved storage: parent offsets (:103)");
            for (uint64_t b = 0; b < nb; b++)
                for (uint64_t i = 0; i < sz; i++) to[base + i + b * sz] = base + b + i * nb;
            base += nb * sz;
        }
        GS_CHECK(base == n, "interleaved storage: parents do not cover the nonzeros");
    }
    return to;
}

void modify_col_indices_by_interlance_storage::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &c = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
    auto to = interlance_storage_permutation(m, parent_pos, target_matrix_id, check);
    std::vector<uint64_t> out(c.size());
    for (uint64_t e = 0; e < c.size(); e++) out[to[e]] = c[e];
    replace_u(GLOBAL_META, "nz_col_indices_after_interlance_storage", std::move(out));
    src(GLOBAL_META, "nz_col_indices");
    src(parent_pos, "BMT_size_of_each_blk");
    is_run = true;
}

void modify_row_indices_by_interlance_storage::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &r = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    auto to = interlance_storage_permutation(m, parent_pos, target_matrix_id, check);
    std::vector<uint64_t> out(r.size());
    for (uint64_t e = 0; e < r.size(); e++) out[to[e]] = r[e];
    replace_u(GLOBAL_META, "nz_row_indices_after_interlance_storage", std::move(out));
    src(GLOBAL_META, "nz_row_indices");
    src(parent_pos, "BMT_size_of_each_blk");
    is_run = true;
}

// modify_vals_by_interlance_storage.cc:69/109/125-135: same permutation, the value type kept
void modify_vals_by_interlance_storage::run(bool check) {
    auto &m = *meta_data_set_ptr;
    auto varr = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
    auto to = interlance_storage_permutation(m, parent_pos, target_matrix_id, check);
    std::vector<double> out(varr->get_len());
    for (uint64_t e = 0; e < out.size(); e++) out[to[e]] = varr->read_float_from_arr(e);
    replace_f(GLOBAL_META, "nz_vals_after_interlance_storage", std::move(out), varr->get_data_type());
    src(GLOBAL_META, "nz_vals");
    src(parent_pos, "BMT_size_of_each_blk");
    is_run = true;
}

// ------------------------------------------------- relative indices (§8f rank 1)
// get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB.cc:45-70:
// per BMTB, its BMW starts minus the BMTB's first row (no ending entry)
void get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &tb = m.u(TBLOCK_META, "first_row_indices", target_matrix_id);
    GS_CHECK(fixed_row_block_size > 0, "fixed_row_block_size > 0");
    std::vector<uint64_t> out;
    for (size_t i = 0; i + 1 < tb.size(); i++)
        for (uint64_t r = tb[i]; r < tb[i + 1]; r += (uint64_t)fixed_row_block_size) out.push_back(r - tb[i]);
    replace_u(WARP_META, "first_row_indices_relative_to_BMTB", std::move(out));
    src(TBLOCK_META, "first_row_indices");
    is_run = true;
}

// get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB.cc:50-85:
// per BMTB, the nonzeros before each BMW counted from the BMTB's first row
void get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &tb = m.u(TBLOCK_META, "first_row_indices", target_matrix_id);
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    const uint64_t row_num = row_num_of_sub_matrix(m, target_matrix_id);
    auto cnt = get_nnz_of_each_row_in_spec_range(row, 0, row_num - 1, 0, row.size() - 1);
    GS_CHECK(fixed_row_block_size > 0, "fixed_row_block_size > 0");
    std::vector<uint64_t> out;
    for (size_t i = 0; i + 1 < tb.size(); i++) {
        uint64_t nz = 0;
        for (uint64_t r = tb[i]; r < tb[i + 1]; r++) {
            if ((r - tb[i]) % (uint64_t)fixed_row_block_size == 0) out.push_back(nz);
            nz += r < cnt.size() ? cnt[r] : 0;
        }
    }
    replace_u(WARP_META, "first_nz_indices_relative_to_BMTB", std::move(out));
    src(TBLOCK_META, "first_row_indices");
    src(GLOBAL_META, "nz_row_indices");
    is_run = true;
}

// ------------------------------------------------ row division (§8f rank 3)
// modify_row_start_boundary_after_fixed_div_in_row_direction.cc:31-75 (and the other six):
// bins of fixed_row_gap_size rows over [begin_row_index, end_row_index]; a bin is
// non-empty when a nonzero's (relative) row falls in it; each transform appends one new
// sub-matrix per non-empty bin, its id = (max existing id of that item) + 1
static std::vector<uint64_t> row_div_bins(const meta_data_set &m, int s, uint64_t gap) {
    GS_CHECK(gap > 0, "fixed_row_gap_size > 0");
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", s), e = m.scalar(GLOBAL_META, "end_row_index", s);
    const uint64_t row_num = e - b + 1;
    const uint64_t nbin = (row_num + gap - 1) / gap;
    std::vector<uint8_t> used(nbin, 0);
    for (uint64_t r : m.u(GLOBAL_META, "nz_row_indices", s)) {
        GS_CHECK(r / gap < nbin, "row division: a nonzero lies past end_row_index");
        used[r / gap] = 1;
    }
    std::vector<uint64_t> bins;
    for (uint64_t i = 0; i < nbin; i++)
        if (used[i]) bins.push_back(i);
    return bins;
}

static void add_scalar_next(meta_data_set &m, POS_TYPE pos, const char *name, uint64_t v) {
    m.add_scalar(pos, name, m.get_max_sub_matrix_id_of_data_item(pos, name) + 1, v);
}

void modify_row_start_boundary_after_fixed_div_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", target_matrix_id);
    for (uint64_t i : row_div_bins(m, target_matrix_id, fixed_row_gap_size))
        add_scalar_next(m, GLOBAL_META, "begin_row_index", b + i * fixed_row_gap_size);
    is_run = true;
}

void modify_row_end_boundary_after_fixed_div_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", target_matrix_id);
    const uint64_t e = m.scalar(GLOBAL_META, "end_row_index", target_matrix_id);
    for (uint64_t i : row_div_bins(m, target_matrix_id, fixed_row_gap_size))
        add_scalar_next(m, GLOBAL_META, "end_row_index", std::min(b + (i + 1) * fixed_row_gap_size - 1, e));
    is_run = true;
}

void modify_col_start_boundary_after_fixed_div_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t c = m.scalar(GLOBAL_META, "begin_col_index", target_matrix_id);
    for (size_t n = row_div_bins(m, target_matrix_id, fixed_row_gap_size).size(); n; n--)
        add_scalar_next(m, GLOBAL_META, "begin_col_index", c);
    is_run = true;
}

void modify_col_end_boundary_after_fixed_div_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t c = m.scalar(GLOBAL_META, "end_col_index", target_matrix_id);
    for (size_t n = row_div_bins(m, target_matrix_id, fixed_row_gap_size).size(); n; n--)
        add_scalar_next(m, GLOBAL_META, "end_col_index", c);
    is_run = true;
}

// fixed_div_col_indices_by_corr_row_indices.cc: the cols of each bin in their order, the
// parent's array removed
void fixed_div_col_indices_by_corr_row_indices::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    const auto &col = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
    std::map<uint64_t, std::vector<uint64_t>> per;
    for (size_t e = 0; e < row.size(); e++) per[row[e] / fixed_row_gap_size].push_back(col[e]);
    for (auto &kv : per)
        m.add_element(GLOBAL_META, "nz_col_indices", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_col_indices") + 1,
                      std::make_shared<universal_array>(std::move(kv.second)));
    m.remove_element(GLOBAL_META, "nz_col_indices", target_matrix_id);
    is_run = true;
}

void fixed_div_vals_by_corr_row_indices::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    auto varr = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
    std::map<uint64_t, std::vector<double>> per;
    for (size_t e = 0; e < row.size(); e++) per[row[e] / fixed_row_gap_size].push_back(varr->read_float_from_arr(e));
    for (auto &kv : per)
        m.add_element(GLOBAL_META, "nz_vals", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_vals") + 1,
                      std::make_shared<universal_array>(std::move(kv.second), varr->get_data_type()));
    m.remove_element(GLOBAL_META, "nz_vals", target_matrix_id);
    is_run = true;
}

// fixed_div_row_indices.cc:12-45: rows relative to the bin (row % gap)
void fixed_div_row_indices::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    std::map<uint64_t, std::vector<uint64_t>> per;
    for (uint64_t r : row) per[r / fixed_row_gap_size].push_back(r % fixed_row_gap_size);
    for (auto &kv : per)
        m.add_element(GLOBAL_META, "nz_row_indices", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices") + 1,
                      std::make_shared<universal_array>(std::move(kv.second)));
    m.remove_element(GLOBAL_META, "nz_row_indices", target_matrix_id);
    is_run = true;
}

// ------------------------------------------- row division by row length (§8f rank 3)
// div_row_indices_by_row_nnz.cc:40-95 (the same loop in all seven transforms and in
// row_nz_matrix_div_operator::is_valid_according_to_metadata)
static void row_nz_window_of(uint64_t nz, const row_nz_window &w, uint64_t &low, uint64_t &high) {
    low = 0;
    high = w.nz_gap_size;
    if (nz < w.max_gap) {
        while (nz >= high && high <= w.max_gap) {
            low = high;
            high *= w.expansion_rate;
        }
    } else {
        low = w.max_gap;
        high = low * w.expansion_rate;
    }
}

std::vector<uint64_t> row_nz_div_positions(const std::vector<uint64_t> &nnz, const row_nz_window &w, size_t max_count,
                                           bool *over) {
    std::vector<uint64_t> div{0};
    if (over) *over = false;
    uint64_t low, high;
    row_nz_window_of(nnz[0], w, low, high);
    for (uint64_t r = 1; r < nnz.size(); r++) {
        const uint64_t nz = nnz[r];
        if ((nz >= low && nz < high) || (nz >= high && high > w.max_gap)) continue;
        div.push_back(r);
        if (max_count && div.size() > max_count) {
            if (over) *over = true;
            break;
        }
        row_nz_window_of(nz, w, low, high);
    }
    return div;
}

static std::vector<uint64_t> row_nz_positions_of(const meta_data_set &m, int s, const row_nz_window &w) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const uint64_t rn = m.scalar(GLOBAL_META, "end_row_index", s) - m.scalar(GLOBAL_META, "begin_row_index", s) + 1;
    GS_CHECK(!row.empty(), "row-length division of an empty sub-matrix");
    return row_nz_div_positions(get_nnz_of_each_row_in_spec_range(row, 0, rn - 1, 0, row.size() - 1), w);
}

// div_row_indices_by_row_nnz.cc:96-125: entries walk the buckets in row order, moving on
// by ONE bucket whenever a row reaches the current bucket's upper bound (the last bucket's
// bound is the last row + 1); rows keep the parent's indexing
template <class T, class F>
static std::vector<std::vector<T>> row_nz_buckets(const std::vector<uint64_t> &row, const std::vector<uint64_t> &div,
                                                  F value_of) {
    std::vector<std::vector<T>> b(div.size());
    size_t cur = 0;
    for (size_t i = 0; i < row.size(); i++) {
        const uint64_t r = row[i];
        const int64_t upper = cur < div.size() - 1 ? (int64_t)div[cur + 1] : (int64_t)row.back() + 1;
        if (r >= div[cur] && (int64_t)r < upper) {
            b[cur].push_back(value_of(i));
        } else if ((int64_t)r >= upper) {
            cur++;
            b[cur].push_back(value_of(i));
        }
    }
    return b;
}

void modify_row_start_boundary_after_div_according_to_row_nz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    for (uint64_t d : row_nz_positions_of(m, target_matrix_id, win)) add_scalar_next(m, GLOBAL_META, "begin_row_index", d);
    is_run = true;
}

void modify_row_end_boundary_after_div_according_to_row_nz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    std::vector<uint64_t> div = row_nz_positions_of(m, target_matrix_id, win);
    div.push_back(m.scalar(GLOBAL_META, "end_row_index", target_matrix_id) -
                  m.scalar(GLOBAL_META, "begin_row_index", target_matrix_id) + 1);
    for (size_t i = 1; i < div.size(); i++) add_scalar_next(m, GLOBAL_META, "end_row_index", div[i] - 1);
    is_run = true;
}

void modify_col_start_boundary_after_div_according_to_row_nz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t c = m.scalar(GLOBAL_META, "begin_col_index", target_matrix_id);
    for (size_t n = row_nz_positions_of(m, target_matrix_id, win).size(); n; n--)
        add_scalar_next(m, GLOBAL_META, "begin_col_index", c);
    is_run = true;
}

void modify_col_end_boundary_after_div_according_to_row_nz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const uint64_t c = m.scalar(GLOBAL_META, "end_col_index", target_matrix_id);
    for (size_t n = row_nz_positions_of(m, target_matrix_id, win).size(); n; n--)
        add_scalar_next(m, GLOBAL_META, "end_col_index", c);
    is_run = true;
}

void div_col_indices_by_row_nnz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    const auto &col = m.u(GLOBAL_META, "nz_col_indices", target_matrix_id);
    auto b = row_nz_buckets<uint64_t>(row, row_nz_positions_of(m, target_matrix_id, win), [&](size_t i) { return col[i]; });
    for (auto &v : b)
        if (!v.empty())
            m.add_element(GLOBAL_META, "nz_col_indices", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_col_indices") + 1,
                          std::make_shared<universal_array>(std::move(v)));
    m.remove_element(GLOBAL_META, "nz_col_indices", target_matrix_id);
    is_run = true;
}

void div_val_indices_by_row_nnz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    auto varr = m.get_element(GLOBAL_META, "nz_vals", target_matrix_id)->meta_data_arr;
    auto b = row_nz_buckets<double>(row, row_nz_positions_of(m, target_matrix_id, win),
                                    [&](size_t i) { return varr->read_float_from_arr(i); });
    for (auto &v : b)
        if (!v.empty())
            m.add_element(GLOBAL_META, "nz_vals", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_vals") + 1,
                          std::make_shared<universal_array>(std::move(v), varr->get_data_type()));
    m.remove_element(GLOBAL_META, "nz_vals", target_matrix_id);
    is_run = true;
}

void div_row_indices_by_row_nnz::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", target_matrix_id);
    auto b = row_nz_buckets<uint64_t>(row, row_nz_positions_of(m, target_matrix_id, win), [&](size_t i) { return row[i]; });
    for (auto &v : b)
        if (!v.empty())
            m.add_element(GLOBAL_META, "nz_row_indices", m.get_max_sub_matrix_id_of_data_item(GLOBAL_META, "nz_row_indices") + 1,
                          std::make_shared<universal_array>(std::move(v)));
    m.remove_element(GLOBAL_META, "nz_row_indices", target_matrix_id);
    is_run = true;
}

// ------------------------------------------ BMT row blocking inside parents (§8f rank 1)
static const char *parent_tag(POS_TYPE p) { return p == TBLOCK_META ? "BMTB" : "BMW"; }

// get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_in_BMTB.cc:30-75 (the _in_BMW
// file is the same over WARP_META): BMT starts first + k*rb inside every parent, then row_num
void get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_in_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &pr = m.u(parent, "first_row_indices", target_matrix_id);
    std::vector<uint64_t> out;
    for (size_t j = 0; j + 1 < pr.size(); j++)
        for (uint64_t r = pr[j]; r < pr[j + 1]; r += (uint64_t)fixed_row_block_size) out.push_back(r);
    out.push_back(row_num_of_sub_matrix(m, target_matrix_id));
    m.add_element(THREAD_META, "first_row_indices", target_matrix_id, std::make_shared<universal_array>(std::move(out)));
    is_run = true;
}

// ..._relative_to_BMTB.cc:30-70: the same starts minus the parent's first row, no end entry
void get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &pr = m.u(parent, "first_row_indices", target_matrix_id);
    std::vector<uint64_t> out;
    for (size_t j = 0; j + 1 < pr.size(); j++)
        for (uint64_t r = pr[j]; r < pr[j + 1]; r += (uint64_t)fixed_row_block_size) out.push_back(r - pr[j]);
    m.add_element(THREAD_META, std::string("first_row_indices_relative_to_") + parent_tag(parent), target_matrix_id,
                  std::make_shared<universal_array>(std::move(out)));
    is_run = true;
}

// get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_in_BMTB.cc:35-85: every parent
// opens a BMT at its first nz (an empty parent included); a new BMT after each rb rows that
// do not end the parent; then the parents' last nz
static std::vector<uint64_t> bmt_nzs_in_parent(meta_data_set &m, int s, POS_TYPE parent, int rb, bool relative) {
    const auto &row = m.u(GLOBAL_META, "nz_row_indices", s);
    const uint64_t rn = row_num_of_sub_matrix(m, s);
    const std::vector<uint64_t> cnt = get_nnz_of_each_row_in_spec_range(row, 0, rn - 1, 0, row.size() - 1);
    const auto &pr = m.u(parent, "first_row_indices", s);
    const auto &pz = m.u(parent, "first_nz_indices", s);
    std::vector<uint64_t> out;
    for (size_t j = 0; j + 1 < pr.size(); j++) {
        const uint64_t base = relative ? 0 : pz[j];
        int rc = 0;
        uint64_t nz = 0;
        out.push_back(base);
        for (uint64_t i = pr[j]; i < pr[j + 1]; i++) {
            rc += 1;
            nz += cnt[i];
            if (rc == rb && i != pr[j + 1] - 1) {
                out.push_back(base + nz);
                rc = 0;
            }
        }
    }
    if (!relative) out.push_back(pz.back());
    return out;
}

void get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_in_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    m.add_element(THREAD_META, "first_nz_indices", target_matrix_id,
                  std::make_shared<universal_array>(bmt_nzs_in_parent(m, target_matrix_id, parent, fixed_row_block_size, false)));
    is_run = true;
}

void get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent::run(bool check) {
    auto &m = *meta_data_set_ptr;
    m.add_element(THREAD_META, std::string("first_nz_indices_relative_to_") + parent_tag(parent), target_matrix_id,
                  std::make_shared<universal_array>(bmt_nzs_in_parent(m, target_matrix_id, parent, fixed_row_block_size, true)));
    is_run = true;
}

// get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction.cc:25-75: per parent the
// index of its first BMT (BMTs counted while their first row lies before the next parent's)
void get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction::run(bool check) {
    auto &m = *meta_data_set_ptr;
    const auto &bt = m.u(THREAD_META, "first_row_indices", target_matrix_id);
    const auto &pr = m.u(parent, "first_row_indices", target_matrix_id);
    std::vector<uint64_t> out{0};
    size_t cur = 0;
    for (size_t j = 0; j + 1 < pr.size(); j++) {
        if (check) GS_CHECK(cur < bt.size() && bt[cur] == pr[j], "a parent does not start with a BMT");
        uint64_t n = 0;
        while (cur < bt.size() && bt[cur] < pr[j + 1]) {
            n++;
            cur++;
        }
        out.push_back(out.back() + n);
    }
    m.add_element(parent, "first_BMT_indices", target_matrix_id, std::make_shared<universal_array>(std::move(out)));
    is_run = true;
}

}  // namespace gs
