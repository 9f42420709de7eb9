// code_generator.hpp -- kernel IR and HIP emission for gfx950.
//
// Reference: code_generator.hpp:44-457, kernel_generator.h (token IR),
// reduction_token/*.cc.  The reference assembles a CUDA kernel from string
// tokens per opened level.  Here the operators attach *reduction tokens*
// (descriptors) to the levels exactly as before (set_reduction_token /
// open_spec_level_of_paral / set_thread_grid), and compile() lowers that
// token set onto one of the hand-written gfx950 kernel families in
// hip_code/kernel_lib.hpp, producing a kernel_spec.  generate_final_program()
// emits a standalone HIP program (kernel_file.hip + plan files +
// make_kernel.sh) that instantiates the same family, with the reference's
// perf_result contract (code_generator.cc:643-648).
#pragma once

#include "gs_core.hpp"

#include <array>
#include <set>

namespace gs {

// reduction tokens the operators attach (reduction_token/*.cc)
enum class reduction_kind {
    NONE,
    TOTAL_BMT_RESULT,      // total_BMT_result_reduce_to_one_register_token (K1)
    THREAD_BIT_MAP,        // thread_bit_map_reduce_to_two_register_token (K2)
    TOTAL_WARP_RESULT,     // total_warp_result_reduce_to_one_register_token (K4)
    WARP_SEGMENT,          // warp_segment_reduce_token (K3)
    TOTAL_BLOCK_RESULT,    // total_block_reduce_to_one_register_token (K6)
    WARP_BIT_MAP,          // warp_bit_map_reduce_token (K5)
    TBLOCK_BIT_MAP,        // tblock_bit_map_reduce_token (K7)
};
const char *reduction_kind_name(reduction_kind k);

struct reduction_token {
    reduction_kind kind = reduction_kind::NONE;
    int coarsen_factor = 1;
    int sparse_coarsen_factor = 1;
    bool need_warp_reduction = false;
    int size = 0;  // VECTOR_WIDTH / bitmap group size
};

// gfx950 kernel families (hip_code/kernel_lib.hpp)
enum kernel_family : int {
    KF_NONE = 0,
    KF_THREAD_TOTAL = 1,    // lane group per BMT row (row-sorted, col-padded)
    KF_WARP_TOTAL = 2,      // one 64-lane wave per BMW (row block), nnz split over lane slots
    KF_BLOCK_TOTAL = 3,     // one workgroup per BMTB row block, LDS reduction
    KF_BITMAP_SEGMENT = 4,  // fixed-nnz BMTs, bitmap row segments, wave-level carry combine
    KF_ROW_CHUNKS = 5,      // col-direction BMTs (chunks of one row), segmented slot tree + row carry
    KF_MERGE_PATH = 6,      // merge-path levels (A11): nz-balanced wave ranges, row-start flags, carries + fix-up
};
const char *kernel_family_name(int f);

struct kernel_spec {
    int family = KF_NONE;
    int coarsen_factor = 1;
    int sparse_coarsen_factor = 1;
    int vector_width = 1;
    bool warp_segment = false;   // K3 present on top of K2
    bool tblock_parent = false;  // BMWs grouped into BMTBs
    bool row_sorted = false;     // GLOBAL original_nz_row_indices present
    POS_TYPE bitmap_parent = THREAD_META;  // K5 (WARP) / K7 (TBLOCK) on col-direction BMTs
    POS_TYPE merge_level = GLOBAL_META;    // merge-path plans: the level the operator split
    int work_size = 0;                     // merge-path plans: path steps per level
    POS_TYPE group_level = WARP_META;      // KF_WARP_TOTAL: level whose first_row_indices are the row groups
    bool interleaved = false;              // cols / vals in interleaved storage
    int interleave_parent = 0;             // ... per GLOBAL_META (one run of BMTs) or per TBLOCK / WARP parent
    std::array<unsigned, 2> ref_grid{{0, 0}}, ref_block{{0, 0}};
    std::vector<std::string> arrays;  // metadata keys the kernel consumes (= kernel arguments)
    std::string name() const;
};

class code_generator {
  public:
    code_generator(std::shared_ptr<meta_data_set> m, int sub_matrix_id);
    std::shared_ptr<meta_data_set> get_metadata_set() const { return meta; }
    int get_sub_matrix_id() const { return sub; }

    void open_spec_level_of_paral(POS_TYPE pos) { opened.insert(pos); }
    bool level_is_open(POS_TYPE pos) const { return opened.count(pos) != 0; }
    // code_generator.cc:2451-2485: one token per level
    void set_reduction_token(POS_TYPE pos, const reduction_token &tok);
    bool reduction_token_is_existing(POS_TYPE pos) const { return tokens.count(pos) != 0; }
    const reduction_token &get_reduction_token(POS_TYPE pos) const { return tokens.at(pos); }
    void set_thread_for_row(bool v) { thread_for_row = v; }
    bool get_thread_for_row() const { return thread_for_row; }
    // merge_path_*_operator: which level holds the merge-path split (the reference opens
    // TBLOCK for all three, so the level is recorded separately)
    void set_merge_path_level(POS_TYPE pos, int work_size) { merge_level = pos; merge_work_size = work_size; }
    // interlance_storage_operator (code_generator.hpp set_interleave_storage): kernels read
    // the *_after_interlance_storage arrays
    void set_interleave_storage(POS_TYPE parent) { interleave = true; interleave_parent = parent; }
    void set_thread_grid(const std::vector<unsigned> &grid, const std::vector<unsigned> &block);

    // lowers the token set to a kernel family (code_generator.hpp:265-269)
    void compile();
    bool is_compiled() const { return compiled; }
    // a plan file's spec (plan_io.cc): the selection compile() made when the plan was saved
    void restore_compiled(const kernel_spec &s) { spec = s; compiled = true; }
    const kernel_spec &get_kernel_spec() const { return spec; }

    // HIP source of the generated program (kernel + main with perf_result).  fp16 plans whose
    // device kernel is a matrix-core one (device_layout.hpp) launch that kernel on the layout
    // arrays generate_final_program writes next to the plan arrays
    std::string generate_kernel_file_source(int repeat) const;
    // writes ROOT/data_source/<id>/{plan arrays, kernel_file.hip, make_kernel.sh}
    // (code_generator.hpp:271-280); returns the id, optionally the directory
    uint64_t generate_final_program(int repeat, const std::string &root, std::string *dir_out = nullptr);

  private:
    std::string generate_gather_source(int repeat) const;  // the CUDA-core families' program
    std::shared_ptr<meta_data_set> meta;
    int sub;
    std::set<POS_TYPE> opened;
    std::map<POS_TYPE, reduction_token> tokens;
    bool thread_for_row = false;
    POS_TYPE merge_level = GLOBAL_META;
    int merge_work_size = 0;
    bool interleave = false;
    POS_TYPE interleave_parent = GLOBAL_META;
    std::vector<unsigned> grid, block;
    bool compiled = false;
    kernel_spec spec;
};

}  // namespace gs
