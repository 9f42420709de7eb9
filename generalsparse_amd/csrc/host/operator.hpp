// operator.hpp -- the plugin surface (operator.hpp:16-1324 of the reference).
//
// Same class names, stages and constructor argument order as the reference
// (the token_test pipelines are written against them); validity is decided
// by the same name-substring rules over the operator history.  run() calls
// the transform steps in data_transform_step.hpp and attaches reduction
// tokens to the code generator.
#pragma once

#include "code_generator.hpp"
#include "data_transform_step.hpp"

namespace gs {

enum OPERATOR_STAGE_TYPE { CONVERTING_OP, DISTRIBUTING_OP, IMPLEMENTING_OP, NONE_OP };
std::string convert_operator_stage_type_to_string(OPERATOR_STAGE_TYPE t);

class basic_operator;

// operator.hpp:191-265: CONVERTING is a flat list, the others per sub-matrix
class operator_context {
  public:
    void add(const std::shared_ptr<basic_operator> &op);
    std::vector<std::shared_ptr<basic_operator>> read_operator_context_arr(OPERATOR_STAGE_TYPE stage, int sub) const;

  private:
    std::vector<std::shared_ptr<basic_operator>> converting;
    std::map<int, std::vector<std::shared_ptr<basic_operator>>> distributing, implementing;
};

class basic_operator {
  public:
    basic_operator(std::string name, std::shared_ptr<meta_data_set> m, OPERATOR_STAGE_TYPE stage, int target_matrix_id)
        : name(std::move(name)), meta_data_set_ptr(std::move(m)), stage(stage), target_matrix_id(target_matrix_id) {}
    virtual ~basic_operator() = default;
    virtual void run(bool check = true) = 0;
    virtual bool is_valid_according_to_metadata() = 0;
    virtual bool is_valid_according_to_operator(std::shared_ptr<operator_context> history) = 0;
    virtual std::vector<std::string> get_data_transform_sequence() const { return transform_seq; }
    virtual std::string convert_to_string() const {
        return name + "::{name:\"" + name + "\",stage:" + convert_operator_stage_type_to_string(stage) +
               ",target_matrix_id:" + std::to_string(target_matrix_id) + "}";
    }
    virtual void set_padding_to_false() {}
    const std::string &get_name() const { return name; }
    OPERATOR_STAGE_TYPE get_stage() const { return stage; }
    int get_target_matrix_id() const { return target_matrix_id; }

  protected:
    std::string name;
    std::shared_ptr<meta_data_set> meta_data_set_ptr;
    OPERATOR_STAGE_TYPE stage;
    int target_matrix_id;
    bool is_run = false;
    std::vector<std::string> transform_seq;
    void run_step(basic_data_transform_step &st, bool check) {
        st.run(check);
        transform_seq.push_back(st.convert_to_string());
    }
    bool has(POS_TYPE p, const char *n) const { return meta_data_set_ptr->is_exist(p, n, target_matrix_id); }
};

using cg_ptr = std::shared_ptr<code_generator>;
using ctx_ptr = std::shared_ptr<operator_context>;

// ---------------------------------------------------------------- CONVERTING
class sort_operator : public basic_operator {  // operator/sort_operator.cc
  public:
    sort_operator(cg_ptr cg, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
};

// operator/empty_row_pad_operator.cc: CONVERTING; gives every empty row of the sub-matrix
// one zero entry (before any blocking, not after sort_operator)
class empty_row_pad_operator : public basic_operator {
  public:
    empty_row_pad_operator(cg_ptr cg, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
};

// operator/fixed_interval_row_matrix_div_operator.cc (§8f rank 3): CONVERTING; splits the
// sub-matrix into sub-matrices of fixed_row_interval_size rows (non-empty intervals only)
class fixed_interval_row_matrix_div_operator : public basic_operator {
  public:
    fixed_interval_row_matrix_div_operator(cg_ptr cg, int fixed_row_interval_size, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",fixed_row_interval_size:" + std::to_string(fixed_row_interval_size);
    }
    int fixed_row_interval_size;
    std::vector<int> new_sub_matrix_ids;  // filled by run()
};

// operator/row_nz_matrix_div_operator.cc (§8f rank 3): CONVERTING; splits the sub-matrix
// into row ranges of similar row length (windows from init_row_size_upper_boundary growing by
// expansion_rate up to max_row_size_upper_boundary).  Restated with the reference's
// quirks: every range gets boundaries, only ranges that receive entries get arrays, the
// entries move on one range at a time, and row indices keep the parent's indexing.  The
// executor runs such "parent-indexed" sub-matrices into scratch outputs in the parent's
// row indexing and sums them into C (a row can straddle two of them; capi.cc spmm_all).
class row_nz_matrix_div_operator : public basic_operator {
  public:
    row_nz_matrix_div_operator(cg_ptr cg, int init_row_size_upper_boundary, int max_row_size_upper_boundary,
                               int expansion_rate, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    int init_row_size_upper_boundary, max_row_size_upper_boundary, expansion_rate;
    // filled by run(): the sub-matrices that received arrays, and the row range of the
    // divided sub-matrix their row indices refer to (its begin_row_index and row count)
    std::vector<int> new_sub_matrix_ids;
    uint64_t parent_row_base = 0, parent_rows = 0;
};

// -------------------------------------------------------------- DISTRIBUTING
class fixed_interval_row_direction_tblock_blocking_operator : public basic_operator {
  public:
    fixed_interval_row_direction_tblock_blocking_operator(cg_ptr cg, int fixed_row_block_size, bool is_padding,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override { is_padding = false; }
    int fixed_row_block_size;
    bool is_padding;

  private:
    cg_ptr code_generator_ptr;
};

class fixed_interval_row_direction_warp_blocking_operator : public basic_operator {
  public:
    fixed_interval_row_direction_warp_blocking_operator(cg_ptr cg, int fixed_row_block_size,
                                                        bool row_index_is_relative_to_BMTB,
                                                        bool nz_index_is_relative_to_BMTB, bool is_padding,
                                                        ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override { is_padding = false; }
    int fixed_row_block_size;
    bool row_index_is_relative_to_BMTB, nz_index_is_relative_to_BMTB, is_padding;

  private:
    cg_ptr code_generator_ptr;
};

class fixed_interval_row_direction_thread_blocking_operator : public basic_operator {
  public:
    fixed_interval_row_direction_thread_blocking_operator(cg_ptr cg, int fixed_row_block_size,
                                                          bool row_index_is_relative_to_parent,
                                                          bool nz_index_is_relative_to_parent, bool is_row_padding,
                                                          bool is_col_padding_with_row_max_size_with_empty_row,
                                                          bool is_col_padding_with_col_size, int col_size,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override {
        is_row_padding = false;
        is_col_padding_with_col_size = false;
        is_col_padding_with_row_max_size_with_empty_row = false;
    }
    int fixed_row_block_size;
    bool row_index_is_relative_to_parent, nz_index_is_relative_to_parent, is_row_padding;
    bool is_col_padding_with_row_max_size_with_empty_row, is_col_padding_with_col_size;
    int col_size;
    std::vector<std::shared_ptr<basic_operator>> former_operator;

  private:
    cg_ptr code_generator_ptr;
};

// operator/fixed_interval_nnz_direction_tblock_blocking_operator.cc: DISTRIBUTING; BMTBs of
// nnz_per_BMTB nonzeros (optionally padded to a multiple), first of all distributing operators
class fixed_interval_nnz_direction_tblock_blocking_operator : public basic_operator {
  public:
    fixed_interval_nnz_direction_tblock_blocking_operator(cg_ptr cg, int nnz_per_BMTB, bool nnz_padding,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override { nnz_padding = false; }
    int get_nnz_per_BMTB() const { return nnz_per_BMTB; }
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",nnz_per_BMTB:" + std::to_string(nnz_per_BMTB);
    }
    int nnz_per_BMTB;
    bool nnz_padding;

  private:
    cg_ptr code_generator_ptr;
};

// operator/fixed_interval_nnz_direction_warp_blocking_operator.cc: DISTRIBUTING; BMWs of
// nnz_per_BMW nonzeros, alone or inside nnz-direction BMTBs (a multiple of nnz_per_BMW)
class fixed_interval_nnz_direction_warp_blocking_operator : public basic_operator {
  public:
    fixed_interval_nnz_direction_warp_blocking_operator(cg_ptr cg, int nnz_per_BMW, bool row_index_is_relative_to_parent,
                                                        bool nz_index_is_relative_to_parent, bool nnz_padding,
                                                        ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override { nnz_padding = false; }
    int get_nnz_per_BMW() const { return nnz_per_BMW; }
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",nnz_per_BMW:" + std::to_string(nnz_per_BMW);
    }
    int nnz_per_BMW;
    bool row_index_is_relative_to_parent, nz_index_is_relative_to_parent, nnz_padding;

  private:
    cg_ptr code_generator_ptr;
};

class fixed_interval_nnz_direction_thread_blocking_operator : public basic_operator {
  public:
    fixed_interval_nnz_direction_thread_blocking_operator(cg_ptr cg, int nnz_per_BMT,
                                                          bool row_index_is_relative_to_parent,
                                                          bool nz_index_is_relative_to_parent, bool nnz_padding,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override { nnz_padding = false; }
    int get_nnz_per_BMT() const { return nnz_per_BMT; }
    int nnz_per_BMT;
    bool row_index_is_relative_to_parent, nz_index_is_relative_to_parent, nnz_padding;

  private:
    cg_ptr code_generator_ptr;
};

class balanced_interval_row_direction_warp_blocking_operator : public basic_operator {
  public:
    balanced_interval_row_direction_warp_blocking_operator(cg_ptr cg, int nnz_per_interval,
                                                           bool row_index_is_relative, bool nz_index_is_relative,
                                                           ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    int nnz_per_interval;
    bool row_index_is_relative_to_BMTB, nz_index_is_relative_to_BMTB;

  private:
    cg_ptr code_generator_ptr;
};

// balanced row-direction TBLOCK blocking (operator/balanced_interval_row_direction_tblock_blocking_operator.cc)
class balanced_interval_row_direction_tblock_blocking_operator : public basic_operator {
  public:
    balanced_interval_row_direction_tblock_blocking_operator(cg_ptr cg, int nnz_per_interval, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",nnz_per_interval:" + std::to_string(nnz_per_interval);
    }
    int nnz_per_interval;

  private:
    cg_ptr code_generator_ptr;
};

// balanced row-direction THREAD blocking (operator/balanced_interval_row_direction_thread_blocking_operator.cc)
class balanced_interval_row_direction_thread_blocking_operator : public basic_operator {
  public:
    balanced_interval_row_direction_thread_blocking_operator(cg_ptr cg, int nnz_per_interval,
                                                             bool row_index_is_relative, bool nz_index_is_relative,
                                                             ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",nnz_per_interval:" + std::to_string(nnz_per_interval);
    }
    int nnz_per_interval;
    bool row_index_is_relative_to_parent, nz_index_is_relative_to_parent;

  private:
    cg_ptr code_generator_ptr;
};

// merge-path distribution at one level (operator/merge_path_{tblock,warp,thread}_operator.cc).
// All three open TBLOCK in the reference whatever their level (:118/:131/:133);
// kept, plus the level recorded for the code generator.
class merge_path_operator_base : public basic_operator {
  public:
    merge_path_operator_base(const char *name, POS_TYPE level, cg_ptr cg, int work_size);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",work_size:" + std::to_string(work_size);
    }
    int get_work_size() const { return work_size; }
    int work_size;
    POS_TYPE level;

  protected:
    cg_ptr code_generator_ptr;
};

class merge_path_tblock_operator : public merge_path_operator_base {
  public:
    merge_path_tblock_operator(cg_ptr cg, int work_size, ctx_ptr history);
    bool is_valid_according_to_operator(ctx_ptr h) override;
};

class merge_path_warp_operator : public merge_path_operator_base {
  public:
    merge_path_warp_operator(cg_ptr cg, int work_size, ctx_ptr history);
    bool is_valid_according_to_operator(ctx_ptr h) override;
};

class merge_path_thread_operator : public merge_path_operator_base {
  public:
    merge_path_thread_operator(cg_ptr cg, int work_size, ctx_ptr history);
    bool is_valid_according_to_operator(ctx_ptr h) override;
};

// operator/interlance_storage_operator.cc (§8f rank 2): interleave the nonzeros of the
// equal-size BMTs inside each parent (GLOBAL, or the WARP / TBLOCK level distributed before)
class interlance_storage_operator : public basic_operator {
  public:
    interlance_storage_operator(cg_ptr cg, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    POS_TYPE pos = GLOBAL_META;

  private:
    cg_ptr code_generator_ptr;
};

// operator/fixed_interval_col_direction_thread_blocking_operator.cc (A10): BMTs are
// chunks of fixed_col_block_size nnz along each row
class fixed_interval_col_direction_thread_blocking_operator : public basic_operator {
  public:
    fixed_interval_col_direction_thread_blocking_operator(cg_ptr cg, int fixed_col_block_size,
                                                          bool row_index_is_relative, bool nz_index_is_relative,
                                                          bool is_padding_with_col_size_in_bmt,
                                                          bool is_col_padding_with_row_max_size_without_empty_row,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override {
        is_padding_with_col_size_in_bmt = false;
        is_col_padding_with_row_max_size_without_empty_row = false;
    }
    int fixed_col_block_size;
    bool row_index_is_relative_to_BMTB, nz_index_is_relative_to_BMTB;
    bool row_index_is_relative_to_BMW = false, nz_index_is_relative_to_BMW = false;
    bool is_padding_with_col_size_in_bmt, is_col_padding_with_row_max_size_without_empty_row;
    POS_TYPE padding_pos = GLOBAL_META;
    std::vector<std::shared_ptr<basic_operator>> former_operator;  // distributing ops before it (re-run after padding)

  private:
    cg_ptr code_generator_ptr;
};

// operator/fixed_interval_col_direction_tblock_blocking_operator.cc: DISTRIBUTING; BMTBs are
// chunks of fixed_col_block_size nonzeros of one row (the first distributing operator)
class fixed_interval_col_direction_tblock_blocking_operator : public basic_operator {
  public:
    fixed_interval_col_direction_tblock_blocking_operator(cg_ptr cg, int fixed_col_block_size,
                                                          bool is_padding_with_col_size_in_bmtb,
                                                          bool is_col_padding_with_row_max_size_without_empty_row,
                                                          ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override {
        is_padding_with_col_size_in_bmtb = false;
        is_col_padding_with_row_max_size_without_empty_row = false;
    }
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",fixed_col_block_size:" + std::to_string(fixed_col_block_size);
    }
    int fixed_col_block_size;
    bool is_padding_with_col_size_in_bmtb, is_col_padding_with_row_max_size_without_empty_row;

  private:
    cg_ptr code_generator_ptr;
};

// operator/fixed_interval_col_direction_warp_blocking_operator.cc: DISTRIBUTING; BMWs are
// chunks of fixed_col_block_size nonzeros of one row, alone or inside row-direction BMTBs
class fixed_interval_col_direction_warp_blocking_operator : public basic_operator {
  public:
    fixed_interval_col_direction_warp_blocking_operator(cg_ptr cg, int fixed_col_block_size,
                                                        bool row_index_is_relative_to_BMTB, bool nz_index_is_relative_to_BMTB,
                                                        bool is_padding_with_col_size_in_bmw,
                                                        bool is_col_padding_with_row_max_size_without_empty_row,
                                                        ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    void set_padding_to_false() override {
        is_padding_with_col_size_in_bmw = false;
        is_col_padding_with_row_max_size_without_empty_row = false;
    }
    std::string convert_to_string() const override {
        return basic_operator::convert_to_string() + ",fixed_col_block_size:" + std::to_string(fixed_col_block_size);
    }
    int fixed_col_block_size;
    bool row_index_is_relative_to_BMTB, nz_index_is_relative_to_BMTB;
    bool is_padding_with_col_size_in_bmw, is_col_padding_with_row_max_size_without_empty_row;
    POS_TYPE padding_pos = GLOBAL_META;
    std::vector<std::shared_ptr<basic_operator>> former_operator;

  private:
    cg_ptr code_generator_ptr;
};

// -------------------------------------------------------------- IMPLEMENTING
class thread_total_reduce_operator : public basic_operator {
  public:
    thread_total_reduce_operator(cg_ptr cg, bool need_warp_reduction, int sparse_coarsen_factor, int coarsen_factor,
                                 ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    bool need_warp_reduction;
    int sparse_coarsen_factor, coarsen_factor;

  private:
    cg_ptr code_generator_ptr;
};

class warp_total_reduce_operator : public basic_operator {
  public:
    warp_total_reduce_operator(cg_ptr cg, int coarsen_factor, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    int coarsen_factor;

  private:
    cg_ptr code_generator_ptr;
};

class tblock_total_reduce_operator : public basic_operator {
  public:
    tblock_total_reduce_operator(cg_ptr cg, int coarsen_factor, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    int coarsen_factor;

  private:
    cg_ptr code_generator_ptr;
};

class thread_bit_map_operator : public basic_operator {
  public:
    thread_bit_map_operator(cg_ptr cg, POS_TYPE pos, unsigned size, unsigned sparse_coarsen_factor,
                            unsigned coarsen_factor, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    POS_TYPE pos;
    unsigned size, sparse_coarsen_factor, coarsen_factor;

  private:
    cg_ptr code_generator_ptr;
};

class warp_segment_reduce_operator : public basic_operator {
  public:
    warp_segment_reduce_operator(cg_ptr cg, unsigned coarsen_factor, bool relative_nz, bool relative_row,
                                 ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    unsigned coarsen_factor;
    bool relative_nz, relative_row;

  private:
    cg_ptr code_generator_ptr;
};

// operator/warp_bit_map_operator.cc (K5): BMWs of VECTOR_WIDTH col-direction BMTs
class warp_bit_map_operator : public basic_operator {
  public:
    warp_bit_map_operator(cg_ptr cg, unsigned coarsen_factor, bool relative_nz, bool relative_row, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    unsigned coarsen_factor;
    bool relative_nz, relative_row;

  private:
    cg_ptr code_generator_ptr;
};

// operator/tblock_thread_bit_map_operator.cc (K7): BMTBs of block_size BMTs
class tblock_thread_bit_map_operator : public basic_operator {
  public:
    tblock_thread_bit_map_operator(cg_ptr cg, unsigned coarsen_factor, int block_size, bool relative_nz,
                                   bool relative_row, ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override;
    bool is_valid_according_to_operator(ctx_ptr h) override;
    unsigned coarsen_factor;
    int block_size;
    bool relative_nz, relative_row;

  private:
    cg_ptr code_generator_ptr;
};

class grid_block_operator : public basic_operator {  // operator/grid_block_operator.cc:2-35
  public:
    grid_block_operator(cg_ptr cg, unsigned grid_x, std::vector<unsigned> block, unsigned coarsen_factor,
                        ctx_ptr history);
    void run(bool check = true) override;
    bool is_valid_according_to_metadata() override { return true; }
    bool is_valid_according_to_operator(ctx_ptr) override { return true; }
    std::vector<unsigned> grid, block;

  private:
    cg_ptr code_generator_ptr;
};

// operator_executer.cc:19-26: assert valid -> run -> record history
class operator_executer {
  public:
    operator_executer() : ctx(std::make_shared<operator_context>()) {}
    void add_and_run(const std::shared_ptr<basic_operator> &op);
    std::shared_ptr<operator_context> get_operator_context() const { return ctx; }
    const std::vector<std::string> &log() const { return history_log; }

  private:
    std::shared_ptr<operator_context> ctx;
    std::vector<std::string> history_log;
};

// data_transform_common.cc:330-376
bool has_row_direction_blocking_in_specific_level(const meta_data_set &m, POS_TYPE pos, int sub);

// Factory used by the C ABI: builds an operator from its reference class name
// and integer arguments (in constructor order, minus cg/history).
std::shared_ptr<basic_operator> make_operator(const std::string &name, const std::vector<long long> &args,
                                              cg_ptr cg, ctx_ptr ctx);

// logical_check.cc: cross-array consistency of the metadata set (metadata_set.cc:806-1890);
// "" when consistent, else the first violation
std::string logical_check(const meta_data_set &m);

}  // namespace gs
