// data_transform_step.hpp -- the atomic plan rewrites on the hot path.
//
// Class names and constructor arguments follow data_transform_step.hpp of the
// reference (one class per transform_step/*.cc file).  Each run() is an O(nnz)
// flat-array pass (the reference regroups through vector<vector<>>); the
// resulting arrays are bit-identical (tests/test_plan_parity.py).
#pragma once

#include "gs_core.hpp"

namespace gs {

class basic_data_transform_step {
  public:
    basic_data_transform_step(std::string name, std::shared_ptr<meta_data_set> m, int target_matrix_id)
        : name(std::move(name)), meta_data_set_ptr(std::move(m)), target_matrix_id(target_matrix_id) {}
    virtual ~basic_data_transform_step() = default;
    virtual void run(bool check) = 0;
    virtual std::string convert_to_string() const {
        return name + "::{name:\"" + name + "\",target_matrix_id:" + std::to_string(target_matrix_id) + "}";
    }
    const std::vector<std::string> &get_source_data_item_ptr_in_data_transform_step() const { return source; }
    const std::vector<std::string> &get_dest_data_item_ptr_in_data_transform_step() const { return dest; }
    std::string name;

  protected:
    std::shared_ptr<meta_data_set> meta_data_set_ptr;
    int target_matrix_id;
    bool is_run = false;
    std::vector<std::string> source, dest;
    void src(POS_TYPE p, const char *n) { source.push_back(get_metadata_item_name(p, n, target_matrix_id)); }
    void dst(POS_TYPE p, const char *n) { dest.push_back(get_metadata_item_name(p, n, target_matrix_id)); }
    void replace_u(POS_TYPE p, const char *n, std::vector<uint64_t> v);
    void replace_f(POS_TYPE p, const char *n, std::vector<double> v, data_type t);
};

#define GS_DECLARE_STEP(cls)                                                        \
    class cls : public basic_data_transform_step {                                  \
      public:                                                                       \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id)                 \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id) {}    \
        void run(bool check) override;                                              \
    };

#define GS_DECLARE_STEP_P(cls, ptype, pname)                                         \
    class cls : public basic_data_transform_step {                                  \
      public:                                                                       \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id, ptype pname)    \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), pname(pname) {} \
        void run(bool check) override;                                              \
        ptype pname;                                                                \
    };

// sort_operator (A3, A4)
GS_DECLARE_STEP(get_row_order_by_length)
GS_DECLARE_STEP(reorder_val_by_index)
GS_DECLARE_STEP(reorder_col_by_index)
GS_DECLARE_STEP(reorder_row_by_index)
GS_DECLARE_STEP(remove_empty_row_in_end_of_sub_matrix)

// empty_row_pad_operator: one zero entry per empty row
GS_DECLARE_STEP(modify_col_indices_by_empty_pad_in_submatrix)
GS_DECLARE_STEP(modify_vals_by_empty_pad_in_submatrix)
GS_DECLARE_STEP(modify_row_indices_by_empty_pad_in_submatrix)

// column padding to a multiple of each row size (A6)
GS_DECLARE_STEP_P(modify_col_indices_by_col_pad_in_sub_matrix, int, multiple_of_each_row_size)
GS_DECLARE_STEP_P(modify_vals_by_col_pad_in_sub_matrix, int, multiple_of_each_row_size)
GS_DECLARE_STEP_P(modify_row_indices_by_col_pad_in_sub_matrix, int, multiple_of_each_row_size)

// row padding: the sub-matrix's row count (end - begin + 1) up to a multiple, one zero entry per
// added row (its row index, the last column) -- modify_*_by_row_pad_in_sub_matrix.cc
GS_DECLARE_STEP_P(modify_col_indices_by_row_pad_in_sub_matrix, int, multiple)
GS_DECLARE_STEP_P(modify_vals_by_row_pad_in_sub_matrix, int, multiple)
GS_DECLARE_STEP_P(modify_row_indices_by_row_pad_in_sub_matrix, int, multiple)

// column padding of every row to its parent's longest row (GLOBAL / TBLOCK / WARP parent); empty
// rows too with padding_with_empty_row (the row-direction thread blocking), else they stay empty
#define GS_DECLARE_STEP_MAXPAD(cls)                                                  \
    class cls : public basic_data_transform_step {                                  \
      public:                                                                       \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id, POS_TYPE parent_pos, bool padding_with_empty_row) \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), parent_pos(parent_pos), \
              padding_with_empty_row(padding_with_empty_row) {}                    \
        void run(bool check) override;                                              \
        POS_TYPE parent_pos;                                                        \
        bool padding_with_empty_row;                                                \
    };
GS_DECLARE_STEP_MAXPAD(modify_col_indices_by_col_pad_parent_blk_to_max_row_size)
GS_DECLARE_STEP_MAXPAD(modify_vals_by_col_pad_parent_blk_to_max_row_size)
GS_DECLARE_STEP_MAXPAD(modify_row_indices_by_col_pad_parent_blk_to_max_row_size)

// fixed row-direction blocking (A7, A8, BMW)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMTBs_after_fixed_blocking_in_row_direction, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMTBs_after_fixed_blocking_in_row_direction, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_without_BMTB, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_in_BMTB, int, fixed_row_block_size)
GS_DECLARE_STEP(get_begin_BMWs_of_BMTB_after_blocking_in_row_direction)
// relative indices (§8f rank 1): BMW starts relative to their BMTB
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB, int, fixed_row_block_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_row_direction_relative_to_BMTB, int, fixed_row_block_size)

// fixed nnz-direction blocking (A9)
GS_DECLARE_STEP_P(modify_col_indices_by_nnz_pad, int, nnz_target)
GS_DECLARE_STEP_P(modify_vals_by_nnz_pad, int, nnz_target)
GS_DECLARE_STEP_P(modify_row_indices_by_nnz_pad, int, nnz_target)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMT)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMT)

// nnz-direction BMW / BMTB blocking and BMTs inside them
// (fixed_interval_nnz_direction_{warp,tblock,thread}_blocking_operator.cc): a unit starts every
// nnz_per_* nonzeros; its row is the row of that nonzero; the row array ends with the row
// count; indices relative to the parent subtract the parent's first row / first nonzero
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMW)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMW)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB, int, nnz_per_BMW)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_nnz_direction_relative_to_BMTB, int, nnz_per_BMW)
GS_DECLARE_STEP_P(get_begin_rows_of_BMTB_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMTB)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMTB_after_fixed_blocking_in_nnz_direction, int, nnz_per_BMTB)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB, int, nnz_per_BMT)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMTB, int, nnz_per_BMT)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW, int, nnz_per_BMT)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_fixed_blocking_in_nnz_direction_relative_to_BMW, int, nnz_per_BMT)
// children per parent (get_begin_BMWs_of_BMTB_after_blocking.cc,
// get_begin_BMTs_of_specific_parent_after_blocking.cc), the unit sizes
// (get_BMW_size_of_each_parent.cc, get_BMTB_size.cc)
GS_DECLARE_STEP(get_begin_BMWs_of_BMTB_after_blocking)
GS_DECLARE_STEP(get_BMTB_size)
GS_DECLARE_STEP_P(get_BMW_size_of_each_parent, POS_TYPE, parent_pos)
GS_DECLARE_STEP_P(get_begin_BMTs_of_specific_parent_after_blocking, POS_TYPE, parent_pos)

// fixed col-direction blocking (A10): every row cut into chunks of col_size nnz
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction, int, col_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction, int, col_size)
// the same chunks as BMWs / BMTBs (fixed_interval_col_direction_{warp,tblock}_blocking_operator.cc):
// rows without ending, nz starts with ending; relative variants restart per row-direction parent
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction, int, col_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction, int, col_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB, int, col_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_fixed_blocking_in_col_direction_relative_to_BMTB, int, col_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMTB_after_fixed_blocking_in_col_direction, int, col_size)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMTB_after_fixed_blocking_in_col_direction, int, col_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMTB, int, col_size)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_fixed_blocking_in_col_direction_relative_to_BMW, int, col_size)
class get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents : public basic_data_transform_step {
  public:
    get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents(std::shared_ptr<meta_data_set> m,
                                                                                  int target_matrix_id, int col_size,
                                                                                  POS_TYPE parent_pos)
        : basic_data_transform_step("get_begin_nzs_of_BMT_after_fixed_blocking_in_col_direction_relative_to_parents",
                                    std::move(m), target_matrix_id),
          col_size(col_size), parent_pos(parent_pos) {}
    void run(bool check) override;
    int col_size;
    POS_TYPE parent_pos;
};
// remove_item_of_metadata.cc: drop one item (a parent level re-built after padding)
class remove_item_of_metadata : public basic_data_transform_step {
  public:
    remove_item_of_metadata(std::shared_ptr<meta_data_set> m, int target_matrix_id, std::string item_name, POS_TYPE pos)
        : basic_data_transform_step("remove_item_of_metadata", std::move(m), target_matrix_id),
          item_name(std::move(item_name)), pos(pos) {}
    void run(bool check) override;
    std::string item_name;
    POS_TYPE pos;
};

// get_BMT_size_of_each_parent.cc (GLOBAL parent only on the shipped pipelines)
class get_BMT_size_of_each_parent : public basic_data_transform_step {
  public:
    get_BMT_size_of_each_parent(std::shared_ptr<meta_data_set> m, POS_TYPE parent_pos, int target_matrix_id,
                                bool row_direction_blocking)
        : basic_data_transform_step("get_BMT_size_of_each_parent", std::move(m), target_matrix_id),
          parent_pos(parent_pos), row_direction_blocking(row_direction_blocking) {}
    void run(bool check) override;
    POS_TYPE parent_pos;
    bool row_direction_blocking;
};

// thread bitmaps and segment arrays (thread_bit_map_operator.cc:60-101)
class thread_bit_map : public basic_data_transform_step {
  public:
    thread_bit_map(std::shared_ptr<meta_data_set> m, bool parent_flag, int parent_size, int target_matrix_id)
        : basic_data_transform_step("thread_bit_map", std::move(m), target_matrix_id), parent_flag(parent_flag),
          parent_size(parent_size) {}
    void run(bool check) override;
    bool parent_flag;
    int parent_size;
};
class segment_empty_flag : public basic_data_transform_step {
  public:
    segment_empty_flag(std::shared_ptr<meta_data_set> m, POS_TYPE pos, int size, int target_matrix_id)
        : basic_data_transform_step("segment_empty_flag", std::move(m), target_matrix_id), pos(pos), size(size) {}
    void run(bool check) override;
    POS_TYPE pos;
    int size;
};
class segment_empty_row_indices : public basic_data_transform_step {
  public:
    segment_empty_row_indices(std::shared_ptr<meta_data_set> m, POS_TYPE pos, int target_matrix_id)
        : basic_data_transform_step("segment_empty_row_indices", std::move(m), target_matrix_id), pos(pos) {}
    void run(bool check) override;
    POS_TYPE pos;
};
class segment_offset : public basic_data_transform_step {
  public:
    segment_offset(std::shared_ptr<meta_data_set> m, bool parent_flag, int size, int target_matrix_id)
        : basic_data_transform_step("segment_offset", std::move(m), target_matrix_id), parent_flag(parent_flag),
          size(size) {}
    void run(bool check) override;
    bool parent_flag;
    int size;
};
class segment_ptr : public basic_data_transform_step {
  public:
    segment_ptr(std::shared_ptr<meta_data_set> m, POS_TYPE pos, int target_matrix_id)
        : basic_data_transform_step("segment_ptr", std::move(m), target_matrix_id), pos(pos) {}
    void run(bool check) override;
    POS_TYPE pos;
};

// warp_segment_reduce_operator.cc:74-111 (merge VW BMTs into a BMW)
#define GS_DECLARE_MERGE(cls)                                                                   \
    class cls : public basic_data_transform_step {                                              \
      public:                                                                                   \
        cls(std::shared_ptr<meta_data_set> m, POS_TYPE pos, int merge_num, int target_matrix_id) \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), pos(pos), merge_num(merge_num) {} \
        void run(bool check) override;                                                          \
        POS_TYPE pos;                                                                           \
        int merge_num;                                                                          \
    };
GS_DECLARE_MERGE(get_begin_rows_after_merge_thread)
GS_DECLARE_MERGE(get_begin_nzs_after_merge_thread)
GS_DECLARE_MERGE(get_begin_BMTs_after_merge_thread)
GS_DECLARE_MERGE(get_begin_rows_relative_to_parent_after_merge_thread)
GS_DECLARE_MERGE(get_begin_nzs_relative_to_parent_after_merge_thread)

// parent_bit_map_of_thread.cc (warp_bit_map_operator.cc / tblock_thread_bit_map_operator.cc)
class parent_bit_map_of_thread : public basic_data_transform_step {
  public:
    parent_bit_map_of_thread(std::shared_ptr<meta_data_set> m, POS_TYPE pos, int target_matrix_id)
        : basic_data_transform_step("parent_bit_map_of_thread", std::move(m), target_matrix_id), pos(pos) {}
    void run(bool check) override;
    POS_TYPE pos;
};

// balanced row-direction warp blocking (A11; data_transform_common.cc:934-989)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)
// balanced BMTs inside a BMTB / BMW parent: get_begin_{rows,nzs}_of_BMT_after_nnz_blocking_in_row_
// direction_{in,relative_to}_{BMTB,BMW}.cc (one class per array, the parent level a parameter)
#define GS_DECLARE_STEP_BAL(cls)                                                     \
    class cls : public basic_data_transform_step {                                  \
      public:                                                                       \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id, POS_TYPE parent_pos, uint64_t nnz_per_interval) \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), parent_pos(parent_pos), \
              nnz_per_interval(nnz_per_interval) {}                                \
        void run(bool check) override;                                              \
        POS_TYPE parent_pos;                                                        \
        uint64_t nnz_per_interval;                                                  \
    };
GS_DECLARE_STEP_BAL(get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_in_parent)
GS_DECLARE_STEP_BAL(get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent)
GS_DECLARE_STEP_BAL(get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_in_parent)
GS_DECLARE_STEP_BAL(get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction_relative_to_parent)
// ... BMWs inside BMTBs (balanced_interval_row_direction_warp_blocking_operator.cc:165-207)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_rows_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_in_BMTB, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMW_after_nnz_blocking_in_row_direction_relative_to_BMTB, uint64_t, nnz_per_interval)

// balanced row-direction TBLOCK / THREAD blocking without a parent (A11;
// get_begin_{rows,nzs}_of_{BMTB,BMT}_after_nnz_blocking_in_row_direction.cc)
GS_DECLARE_STEP_P(get_begin_rows_of_BMTB_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMTB_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_rows_of_BMT_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)
GS_DECLARE_STEP_P(get_begin_nzs_of_BMT_after_nnz_blocking_in_row_direction, uint64_t, nnz_per_interval)

// merge-path level splits (A11; get_begin_{rows,nzs}_of_level_after_merge_path.cc).
// Constructor order as the reference: (meta, target_matrix_id, pos, work_size).
#define GS_DECLARE_MERGE_PATH(cls)                                                                \
    class cls : public basic_data_transform_step {                                                \
      public:                                                                                     \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id, POS_TYPE pos, int work_size)  \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), pos(pos), work_size(work_size) {} \
        void run(bool check) override;                                                            \
        POS_TYPE pos;                                                                             \
        int work_size;                                                                            \
    };
GS_DECLARE_MERGE_PATH(get_begin_rows_of_level_after_merge_path)
GS_DECLARE_MERGE_PATH(get_begin_nzs_of_level_after_merge_path)

// the merge path of a sub-matrix: level starts every work_size path steps,
// path = one step per nonzero plus one per row change between non-empty rows
// (get_begin_rows_of_level_after_merge_path.cc:58-94); rows / nzs per level
void merge_path_levels(const std::vector<uint64_t> &nnz_of_each_row, uint64_t work_size,
                       std::vector<uint64_t> *level_rows, std::vector<uint64_t> *level_nzs);

// BMT row blocking inside BMTB / BMW parents (§8f rank 1 relative indices;
// get_begin_{rows,nzs}_of_BMT_after_fixed_blocking_in_row_direction_{in,relative_to}_{BMTB,BMW}.cc,
// get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction.cc): BMTs of
// fixed_row_block_size rows start at every parent's first row
#define GS_DECLARE_STEP_POS(cls)                                                                  \
    class cls : public basic_data_transform_step {                                                \
      public:                                                                                     \
        cls(std::shared_ptr<meta_data_set> m, int target_matrix_id, POS_TYPE parent, int fixed_row_block_size) \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), parent(parent),    \
              fixed_row_block_size(fixed_row_block_size) {}                                       \
        void run(bool check) override;                                                            \
        POS_TYPE parent;                                                                          \
        int fixed_row_block_size;                                                                 \
    };
GS_DECLARE_STEP_POS(get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_in_parent)
GS_DECLARE_STEP_POS(get_begin_rows_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent)
GS_DECLARE_STEP_POS(get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_in_parent)
GS_DECLARE_STEP_POS(get_begin_nzs_of_BMT_after_fixed_blocking_in_row_direction_relative_to_parent)
GS_DECLARE_STEP_POS(get_begin_BMTs_of_specific_parent_after_blocking_in_row_direction)

// row division into sub-matrices (§8f rank 3; fixed_interval_row_matrix_div_operator.cc:85-150):
// every non-empty interval of fixed_row_gap_size rows becomes a new sub-matrix (ids max + 1, ...)
GS_DECLARE_STEP_P(modify_row_start_boundary_after_fixed_div_in_row_direction, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(modify_row_end_boundary_after_fixed_div_in_row_direction, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(modify_col_start_boundary_after_fixed_div_in_row_direction, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(modify_col_end_boundary_after_fixed_div_in_row_direction, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(fixed_div_col_indices_by_corr_row_indices, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(fixed_div_vals_by_corr_row_indices, uint64_t, fixed_row_gap_size)
GS_DECLARE_STEP_P(fixed_div_row_indices, uint64_t, fixed_row_gap_size)

// row division by row length (§8f rank 3; row_nz_matrix_div_operator.cc, *_after_div_according_to_row_nz.cc,
// div_{row,col,val}_indices_by_row_nnz.cc): a new sub-matrix starts wherever a row's nnz leaves the
// current window [low, high) (windows grow from nz_gap_size by expansion_rate up to max_gap)
struct row_nz_window {
    uint64_t nz_gap_size, max_gap, expansion_rate;
};
// the division positions (row ids relative to the sub-matrix); max_count > 0 stops after
// more than max_count positions (the operator's validity check) and sets *over
std::vector<uint64_t> row_nz_div_positions(const std::vector<uint64_t> &nnz_of_each_row, const row_nz_window &w,
                                           size_t max_count = 0, bool *over = nullptr);
GS_DECLARE_STEP_P(modify_row_start_boundary_after_div_according_to_row_nz, row_nz_window, win)
GS_DECLARE_STEP_P(modify_row_end_boundary_after_div_according_to_row_nz, row_nz_window, win)
GS_DECLARE_STEP_P(modify_col_start_boundary_after_div_according_to_row_nz, row_nz_window, win)
GS_DECLARE_STEP_P(modify_col_end_boundary_after_div_according_to_row_nz, row_nz_window, win)
GS_DECLARE_STEP_P(div_col_indices_by_row_nnz, row_nz_window, win)
GS_DECLARE_STEP_P(div_val_indices_by_row_nnz, row_nz_window, win)
GS_DECLARE_STEP_P(div_row_indices_by_row_nnz, row_nz_window, win)

// interleaved storage (§8f rank 2; modify_{col,val,row}_indices_by_interlance_storage.cc):
// inside every parent block the i-th nonzero of BMT b moves to b + i * (BMTs in the parent)
#define GS_DECLARE_INTERLANCE(cls)                                                                \
    class cls : public basic_data_transform_step {                                                \
      public:                                                                                     \
        cls(std::shared_ptr<meta_data_set> m, POS_TYPE parent_pos, int target_matrix_id)          \
            : basic_data_transform_step(#cls, std::move(m), target_matrix_id), parent_pos(parent_pos) {} \
        void run(bool check) override;                                                            \
        POS_TYPE parent_pos;                                                                      \
    };
GS_DECLARE_INTERLANCE(modify_col_indices_by_interlance_storage)
GS_DECLARE_INTERLANCE(modify_vals_by_interlance_storage)
GS_DECLARE_INTERLANCE(modify_row_indices_by_interlance_storage)
// the permutation the three transforms apply: new position of old position e
std::vector<uint64_t> interlance_storage_permutation(const meta_data_set &m, POS_TYPE parent_pos, int sub, bool check);

std::vector<uint64_t> get_begin_nzs_of_child_after_balance_blocking_in_row_direction(
    const std::vector<uint64_t> &nnz_of_each_row, uint64_t nnz_per_interval);
std::vector<uint64_t> get_begin_rows_of_child_after_balance_blocking_in_row_direction(
    const std::vector<uint64_t> &nnz_of_each_row, uint64_t nnz_per_interval, uint64_t row_num);

}  // namespace gs
