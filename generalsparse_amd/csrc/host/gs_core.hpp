// gs_core.hpp -- typed arrays, config and the metadata set ("the plan").
//
// Mirrors the reference's L0-L2 interface:
//   data_type enum            struct.hpp:32-70
//   universal_array           code_source_data.hpp / code_source_data.cc:91-461
//   meta_data_item / set      metadata_set.hpp:62-154, metadata_set.cc:147-571
//   get_config / set_config   config.cc:2-40 (re-designed: parsed once, in memory,
//                             thread-safe; a missing key still reads as false/0)
// Storage is redesigned for MI355X-sized inputs: integer arrays are flat
// std::vector<uint64_t> (the reference's UNSIGNED_LONG) and values are a flat
// std::vector<double>; the compressed device types are derived on upload.
#pragma once

#include <cstdint>
#include <map>
#include <memory>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace gs {

// struct.hpp:32-70 (same order, so vector types are base + log2(width))
enum data_type {
    CHAR, UNSIGNED_CHAR, CHAR2, CHAR4, CHAR8,
    SHORT, UNSIGNED_SHORT, SHORT2, SHORT4, SHORT8,
    INT, UNSIGNED_INT, INT2, INT4, NONE_DATA_TYPE_1,
    LONG, UNSIGNED_LONG, LONG2, NONE_DATA_TYPE_2, NONE_DATA_TYPE_3,
    LONG_LONG, UNSIGNED_LONG_LONG,
    HALF, HALF2, HALF4, HALF8,
    FLOAT, FLOAT2, FLOAT4, NONE_DATA_TYPE_4,
    DOUBLE, DOUBLE2, NONE_DATA_TYPE_5, NONE_DATA_TYPE_6,
    BOOL, NONE_DATA_TYPE,
};

std::string code_of_data_type(data_type t);
size_t size_of_data_type(data_type t);
// op_manager.cc:985-1016
data_type find_most_suitable_data_type(uint64_t max_index_number);

// metadata_set.hpp:13-23
enum POS_TYPE { GLOBAL_META, TBLOCK_META, WARP_META, THREAD_META, ROW_META, COL_META, VAL_META, NONE_META };
std::string convert_pos_type_to_string(POS_TYPE t);
std::string get_metadata_item_name(POS_TYPE pos, const std::string &name, int sub_matrix_id);

// All reference `assert`s on the hot path become this exception; the C ABI
// turns it into a negative return code (SURVEY.md §8b "no aborts across the ABI").
struct gs_error : std::runtime_error {
    int code;
    explicit gs_error(const std::string &m, int c = -1) : std::runtime_error(m), code(c) {}
};
#define GS_CHECK(cond, msg) \
    do { if (!(cond)) throw ::gs::gs_error(std::string(msg) + " [" #cond "]"); } while (0)

// ---------------------------------------------------------------- config
// global_config.json.bak keys that the hot path reads.
struct config_t {
    int64_t DENSE_MATRIX_SIZE = 8;
    int64_t VECTOR_WIDTH = 8;
    bool HALF = true;
    std::string PRECISE_OF_FLOAT = "float";
    std::string ROOT_PATH_STR = ".";
    std::string DATA_SET = "";
    bool OPERATOR_RUNTIME_CHECK = true;
    int64_t PADDING_RATE_UP_BOUND = 4;
    bool DATA_TYPE_COMPRESS = true;
    int64_t BRANCH_COMPRESS_MAX_SIZE = 5;
    int64_t FLOAT_RATE = 2;
    double GFLOPS_UP_BOUND = 10000;
    int64_t SHARED_MEM_TOTAL_SIZE = 160 * 1024;  // MI355X LDS per CU
    int64_t MAX_DIV_TIMES_OF_DIV = 12;
    int64_t MFMA_GLDS = 1;  // k_mfma_rows: B rows by global_load_lds (two chunks ahead)
    int64_t MFMA_COMPUTE_WAVES = 6;  // k_mfma_rows compute waves (6, or 8 with two fewer entry waves)
    int64_t MFMA_GLDS_NBUF = 3;  // ... into this many B buffers, NBUF-1 chunks ahead (4, 5: 256-column chunks)
    std::string FORMAT_OF_MTX = "COO";
    std::string PERFORMANCE_FLAG = "throughput";
    std::string Graph_Algorithm = "";
    bool MODEL_DRIVEN_COMPRESS = false;  // absent in the .bak -> false
    // MI355X engine switches (not in the reference)
    bool LDS_STAGE_B = true;  // warp_total inside BMTBs: stage B chunks in LDS (k_lds_rows)
    bool MFMA_TILES = true;   // fp16 BMTB row blocks on the matrix cores (k_mfma_rows)
    int64_t MFMA_KROT = 0;
    int64_t WARP_ROWS_CHUNKS = 3;  // k_warp_rows grouped passes: SCF-chunks per slot in one pass (1..3)
    int64_t WARP_ROWS_GROUPS = 1;  // k_warp_rows: several short rows of a BMW per wave pass    // k_mfma_rows / k_nm_mfma: each workgroup starts at its own K chunk
    int64_t MFMA_MAX_FILL = 16;  // ... when (padded row-block area) / nnz <= this
    bool NM_MFMA = true;         // col-direction plans whose rows are 2:4 panels: sparse matrix cores (k_nm_mfma)
    int64_t MFMA_KSPLIT = 0;     // workgroups per row block (K ranges); 0 = fill the 256 CUs
    bool MFMA_FLAGS = false;     // k_mfma_rows roles hand buffers over through LDS counters
    bool NM_KS = false;          // 2:4 panels: k_nm_mfma_ks (256-row workgroups, K split) instead of k_nm_mfma
                                 // (opt-in: C3 93 us against 66 us, profiles/r03_c3_nmks.json)
    int64_t NM_SPLIT = 0;        // ... its K ranges per row block (0: cover the CUs)
    bool MFMA_BM = false;        // fp16 BMTB row blocks of <= 96 rows: bitmap records, k_mfma_bm
    int64_t BM_SPLIT = 0;        // k_mfma_bm K ranges per row block (0: fill the CUs)
    int64_t BM_WAVES = 8;        // k_mfma_bm waves per workgroup (4 or 8)
    bool BM_KB = false;          // ... k_mfma_kb (k_mfma_ks pipeline on the bitmap layout)
    bool BM_V2 = false;          // ... k_mfma_bm2 (one wave per row tile) when the B slice fits LDS
                                 // (C2 22.9 us against 18.4 for k_mfma_bm, profiles/r03_c2_bm_timeline.json)
    bool MFMA_KS = true;         // row blocks of >= KS_MIN_ROWS rows: K-split, B-stationary k_mfma_ks
    int64_t KS_MIN_ROWS = 40;    // ... from this many rows per BMTB (shorter blocks: k_mfma_rows)
    bool MP_ROWS = false;        // merge-path plans: k_merge_rows (product/row walk) instead of k_merge_path
    int64_t MP_COL_PERM = -1;    // merge-path plans: columns renumbered by degree, B gathered into that order per
                                 // launch (1 on, 0 off, -1 auto: B of at least 64 MB, past the L2s and a quarter
                                 // of the Infinity Cache)
    int64_t MP_PERM_SCATTER = 0; // MP_COL_PERM: B permuted by a scatter (coalesced reads of B rows, rows written to
                                 // their new places) instead of a gather
    int64_t MP_PERM_HOT = 0;     // MP_COL_PERM: 0 = every column sorted by degree; H > 0 = only the H densest columns
                                 // move to the front (by degree), the others keep their order after them
    int64_t MP_SOLO = 16;        // k_merge_rows: rows of at most this many nonzeros are one slot's
    int64_t KS_WAVES = 8;        // k_mfma_ks waves per workgroup (8 or 16)
    int64_t KS_SPLIT = 0;        // k_mfma_ks K ranges per row block (0: the fewest that fit LDS and fill the CUs)
    int64_t NM_V4 = 0;           // 2:4 panels on k_nm_mfma4 (256-row workgroups, K split): 1 at N = 64 / 128, 0 never,
                                 // -1 at N = 128 (K a multiple of 256)
    int64_t KS_POS8 = 0;         // k_mfma_ks at N = 32: 8-bit entry positions in 8 x 16 segments (3 B per nonzero)
    int64_t KS_APART = 1;        // k_mfma_ks: partial tiles beside the wave stages when they fit (1), never (0: the
                                 // stage LDS is reused, more workgroups per CU; N = 32, RT <= 5), or only when that
                                 // keeps the workgroups per CU (-1)
    int64_t KS_FORCE_TIMEOUT = 0;  // experiments build: the K-split combine takes its timeout path (test of the error word)
    int64_t KS_PRIO = 1;         // k_mfma_ks: the younger waves at s_setprio 1 (1: whole loop, 2: first half, 0: off)
    int64_t KS_NT = 0;           // k_mfma_ks at N = 32: A's groups by non-temporal loads; a plan-search variant (C2
                                 // 13.8 -> 12.9 us, the headline layer 165.7 -> 167.8 us; B's rows as well: 14.1 us,
                                 // profiles/r05n_nt3.txt)
    int64_t KS_HEAD = 1;         // k_mfma_ks: the head steps (each wave's first kKsDepth k-steps) at fixed, padded
                                 // places, loaded without their records (when the padding costs <= 6% more groups)
    int64_t KS_PERSIST = 0;      // k_mfma_ks: persistent grid size pulling (row block, K range) units (experiments build)
    int64_t MP_HUB_COLS = 0;     // MP_COL_PARTS = 2: partition 0 = this many densest columns (0: round-robin)
    int64_t MP_COL_PARTS = 0;    // merge path with MP_COL_PERM, fp32: column partitions, one pass each (0/1: off)
    int64_t LDS_DMA = 1;         // k_lds_rows at fp32 N = 32: chunks by LDS-DMA into two buffers (k_lds_rows_dma)
    int64_t LDS_KSPLIT = 0;      // k_lds_rows: workgroups per BMTB, each over a K range (fp32 slab combine; 0 auto)
    int64_t NM_TILES = 0;        // k_nm_mfma: 16-row tiles per workgroup (0: nm_tiles_for; 2, 4, 7, 8)
    int64_t NM_KROT = 1;         // k_nm_mfma: each workgroup walks K from its own 256-row B chunk (C3 -3%,
                                 // profiles/r05ad_krot.txt; 0: every workgroup from chunk 0)
    int64_t NM_NT = 1;           // k_nm_mfma: A's panel blocks by non-temporal loads (C3 at N = 8 / 32 / 128: -10 / -6 /
                                 // -6.5%, profiles/r05n_nt3.txt)
};
// Process-wide config: loaded once from $GS_CONFIG or ./global_config.json if
// present (flat JSON object of scalars), defaults otherwise.
config_t get_config();
void set_config(const std::string &key, int64_t value);
int64_t get_config_int(const std::string &key);  // integer / bool keys
void set_config_str(const std::string &key, const std::string &value);
void reset_config();

// ---------------------------------------------------------------- arrays
class universal_array {
  public:
    universal_array(std::vector<uint64_t> v, data_type t = UNSIGNED_LONG);
    universal_array(std::vector<double> v, data_type t);  // FLOAT or DOUBLE
    uint64_t get_len() const { return is_float_ ? f_.size() : u_.size(); }
    data_type get_data_type() const { return type_; }
    bool is_float() const { return is_float_; }
    uint64_t read_integer_from_arr(uint64_t i) const { return u_[i]; }
    double read_float_from_arr(uint64_t i) const { return is_float_ ? f_[i] : (double)u_[i]; }
    const std::vector<uint64_t> &u() const { return u_; }
    const std::vector<double> &f() const { return f_; }
    std::vector<uint64_t> &u_mut() { return u_; }
    // code_source_data.cc:383-413: smallest unsigned type that holds the max
    data_type get_compress_data_type() const;
    uint64_t max_integer() const;
    // struct.cc:1991-2032: one value per line; floats <= 1e-10 written as 0
    void output_2_file(const std::string &path) const;
    bool check() const { return true; }

  private:
    data_type type_;
    bool is_float_;
    std::vector<uint64_t> u_;
    std::vector<double> f_;
};

struct meta_data_item {
    std::shared_ptr<universal_array> meta_data_arr;
    POS_TYPE meta_position;
    std::string name;
    int sub_matrix_id;
    bool is_constant;
    std::shared_ptr<universal_array> get_metadata_arr() const { return meta_data_arr; }
};

class meta_data_set {
  public:
    std::string matrix_name;
    void add_element(POS_TYPE pos, const std::string &name, int sub, std::shared_ptr<universal_array> arr,
                     bool constant = false);
    void add_scalar(POS_TYPE pos, const std::string &name, int sub, uint64_t v);
    void remove_element(POS_TYPE pos, const std::string &name, int sub);
    void remove_element(const std::string &key);
    std::shared_ptr<meta_data_item> get_element(POS_TYPE pos, const std::string &name, int sub) const;
    std::shared_ptr<meta_data_item> get_element(const std::string &key) const;
    bool is_exist(POS_TYPE pos, const std::string &name, int sub) const;
    bool is_exist(const std::string &key) const { return data_map.count(key) != 0; }
    uint64_t scalar(POS_TYPE pos, const std::string &name, int sub) const {
        return get_element(pos, name, sub)->meta_data_arr->read_integer_from_arr(0);
    }
    const std::vector<uint64_t> &u(POS_TYPE pos, const std::string &name, int sub) const {
        return get_element(pos, name, sub)->meta_data_arr->u();
    }
    int count_of_metadata_of_diff_pos(POS_TYPE pos, int sub) const;
    std::vector<std::string> all_item_of_metadata_of_diff_pos(POS_TYPE pos, int sub) const;
    std::vector<std::string> keys() const;
    // metadata_set.cc get_max_sub_matrix_id_of_data_item: -1 when absent
    int get_max_sub_matrix_id_of_data_item(POS_TYPE pos, const std::string &name) const;
    bool check() const { return true; }
    // metadata_set.cc:517-571 (no sleep(); id from a counter + time)
    uint64_t output_format_to_dir(const std::string &root, const std::vector<std::string> &keys,
                                  std::string *dir_out = nullptr) const;

  private:
    std::map<std::string, std::shared_ptr<meta_data_item>> data_map;
};

// struct.cc:49-261 (A1).  ones_values reproduces the reference (val := 1).
struct coo_t {
    uint64_t max_row_index = 0, max_col_index = 0;
    std::vector<uint64_t> row, col;
    std::vector<float> val;
};
void get_matrix_index_and_val_from_file(const std::string &path, bool ones_values, coo_t &out);

// metadata_set.cc:612-707 (A2) from a file or from in-memory COO arrays.
std::shared_ptr<meta_data_set> create_init_metadata_set_from_file(const std::string &path,
                                                                  const std::string &name, bool ones_values);
std::shared_ptr<meta_data_set> create_init_metadata_set_from_coo(uint64_t n_rows, uint64_t n_cols, uint64_t nnz,
                                                                 const uint64_t *row, const uint64_t *col,
                                                                 const float *val, const std::string &name);

// helpers shared by transforms
// data_transform_common.cc:7-48
std::vector<uint64_t> get_nnz_of_each_row_in_spec_range(const std::vector<uint64_t> &rows, uint64_t begin_row,
                                                        uint64_t end_row, uint64_t begin_nz, uint64_t end_nz);
// the "real end row" rule used by every row-direction transform
uint64_t row_num_of_sub_matrix(const meta_data_set &m, int sub);

}  // namespace gs
