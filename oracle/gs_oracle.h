/*
 * gs_oracle.h -- CPU restatement of GeneralSparse's SpMM hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker for the MI355X
 * engine in generalsparse_amd/.  Only tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg may load it.  The product never links it.
 *
 * Every function restates one reference transform/operator and cites the
 * reference file:line it follows (paths relative to the reference root).
 * Parity pinning: the reference cannot be built or run here (SURVEY.md §8c
 * records the denial), and it ships no fixtures.  The oracle is pinned by
 *   (1) the reference's own known answer: all-ones A and B give
 *       C[i][j] = nnz(row i) exactly (code_generator.cc:633-637,
 *       cuda_code/kernel_lib.hpp:884-921), and
 *   (2) hand-derived plan arrays for small matrices (tests/golden/ JSON files,
 *       derived by reading the cited transforms, see tests/golden/README.md),
 *   (3) the structural invariants the reference asserts.
 */
#ifndef GS_ORACLE_H
#define GS_ORACLE_H

#include <stdint.h>
#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

#define OR_MAX_ARRAYS 128
#define OR_NAME_LEN 96

/* One named plan array: key = "<POS>_<name>_<sub>" (metadata_set.cc:147-151).
 * Integer arrays are stored as u64 (the reference's UNSIGNED_LONG),
 * value arrays as double (read_float_from_arr). */
typedef struct {
    char key[OR_NAME_LEN];
    uint64_t len;
    int is_float;
    uint64_t *u;
    double *f;
} or_array;

typedef struct {
    or_array a[OR_MAX_ARRAYS];
    int n;
    char err[256];
} or_set;

/* COO as read by get_matrix_index_and_val_from_file (struct.cc:49-261). */
typedef struct {
    uint64_t nnz;
    uint64_t *row;
    uint64_t *col;
    float *val;
    uint64_t max_row_index; /* from header (M-1), raised by data */
    uint64_t max_col_index;
} or_coo;

/* A1: .mtx reader.  ones_values=1 reproduces struct.cc:186-200 (val := 1). */
int or_read_mtx(const char *path, int ones_values, or_coo *out);
void or_coo_free(or_coo *c);

/* A2: initial metadata set (metadata_set.cc:612-707). */
int or_init_set(or_set *s, uint64_t n_rows, uint64_t n_cols, uint64_t nnz,
                const uint64_t *row, const uint64_t *col, const float *val);
void or_set_free(or_set *s);
or_array *or_find(or_set *s, const char *key);
int or_count(const or_set *s);
const char *or_key(const or_set *s, int i);
uint64_t or_len(const or_set *s, int i);
int or_is_float(const or_set *s, int i);
const uint64_t *or_u(const or_set *s, int i);
const double *or_f(const or_set *s, int i);
const char *or_error(const or_set *s);

/* Operators (return 0 on success, <0 with s->err on a reference assert). */
int or_sort_operator(or_set *s);                                           /* A3,A4 */
int or_empty_row_pad(or_set *s);                                           /* empty_row_pad_operator */
int or_row_dir_thread_blocking(or_set *s, int rb, int col_pad_size);       /* A5-A7 */
int or_row_dir_tblock_blocking(or_set *s, int rb);                         /* A8 */
int or_row_dir_warp_blocking(or_set *s, int rb);                           /* BMW */
int or_nnz_dir_thread_blocking(or_set *s, int nnz_per_bmt, int pad);       /* A9 */
int or_nnz_dir_tblock_blocking(or_set *s, uint64_t nnz_per_bmtb, int pad); /* nnz-direction BMTBs */
int or_nnz_dir_warp_blocking(or_set *s, uint64_t nnz_per_bmw, int rrel, int nrel, int pad); /* nnz BMWs */
int or_nnz_dir_thread_in_parent(or_set *s, uint64_t nnz_per_bmt, int rrel, int nrel); /* BMTs in them */
int or_thread_bit_map_operator(or_set *s, int pos_is_warp, int size);      /* A9 */
int or_warp_segment_operator(or_set *s, int vw);                           /* A9 */
int or_balanced_row_dir_warp_blocking(or_set *s, uint64_t nnz_per_bmw);    /* A11 */
int or_balanced_row_dir_tblock_blocking(or_set *s, uint64_t nnz_per_bmtb); /* A11 */
int or_balanced_row_dir_thread_blocking(or_set *s, uint64_t nnz_per_bmt);  /* A11 */
int or_merge_path(or_set *s, const char *pos, uint64_t work_size);         /* A11 */
int or_interlance_storage_global(or_set *s);                               /* §8f rank 2 */
int or_bmw_relative_to_bmtb(or_set *s, int rb);                            /* §8f rank 1 */
int or_bmt_in_parent(or_set *s, int rb, int rrel, int nrel);               /* §8f rank 1 */
int or_fixed_interval_row_div(or_set *s, uint64_t gap);                    /* §8f rank 3 */
int or_row_nz_div(or_set *s, uint64_t init, uint64_t max_gap, uint64_t rate); /* §8f rank 3 */
int or_index_compression(const uint64_t *a, uint64_t n, int type_ori, int branch_max, int *kind,
                         uint64_t *params, uint64_t *res);                 /* §8f rank 1 */
int or_col_dir_thread_blocking(or_set *s, int col_size, int pad);          /* A10 */
/* col-direction BMWs / BMTBs and col-direction BMTs inside row-direction parents */
int or_col_dir_tblock_blocking(or_set *s, uint64_t col_size, int pad);
int or_col_dir_warp_blocking(or_set *s, uint64_t col_size, int rrel, int nrel);
int or_col_dir_thread_in_parent(or_set *s, uint64_t col_size, int rrel, int nrel, int pad);
int or_parent_bit_map_operator(or_set *s, int pos_is_warp, int merge, int rel_nz, int rel_row); /* K5/K7 */

/* Canned pipelines = token_test.cc test_spmm_* operator sequences. */
int or_pipeline(or_set *s, const char *name, int p0, int p1);

/* A17: CPU SpMM references.  CSR is built from the ORIGINAL coo (the
 * reference's generated main() checks against the original CSR,
 * code_generator.cc:631-638).  B row-major K x N, C row-major M x N. */
void or_spmm_f64(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                 const uint64_t *col, const float *val, const double *B,
                 double *C);
/* spmm_reference_host (kernel_lib.hpp:859-881) with DType=float. */
void or_spmm_ref_f32(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, const float *B,
                     float *C);
/* Same with DType=half: every product and partial sum is rounded to fp16. */
void or_spmm_ref_f16(uint64_t M, uint64_t N, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, const float *B,
                     float *C);
float or_round_half(float x);

/* cpu_baseline helper: run thread_total transform + f32 reference SpMM,
 * returns seconds for each phase. */
int or_time_cpu_path(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                     const uint64_t *col, const float *val, uint64_t N,
                     double *t_transform, double *t_spmm);

int or_time_spmm_repeated(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                          const uint64_t *col, const float *val, uint64_t N, double min_s,
                          double *t_total, int *reps);
/* the build's all-cores variant (OpenMP over rows; the reference's host path is single-threaded) */
int or_time_spmm_repeated_mt(uint64_t M, uint64_t K, uint64_t nnz, const uint64_t *row,
                             const uint64_t *col, const float *val, uint64_t N, double min_s,
                             int threads, double *t_total, int *reps);

#ifdef __cplusplus
}
#endif
#endif
