/*
 * generalsparse.h -- C ABI of the MI355X-native GeneralSparse SpMM engine.
 *
 * This is the drop-in boundary for the reference's SpMM path.
 * Plain pointers and sizes only; every call returns 0 or a negative error
 * code (gs_last_error() has the message); nothing aborts across the ABI
 * (the reference asserts everywhere).  Reentrant per plan, one HIP stream per
 * call, no internal host threads.
 *
 * Reference interfaces each entry point replaces:
 *   gs_plan_create_from_mtx   create_init_metadata_set_from_file   metadata_set.cc:612-707
 *                             (+ get_matrix_index_and_val_from_file  struct.cc:49-261)
 *   gs_plan_create_from_coo   same, from in-memory COO (no text round trip)
 *   gs_plan_add_operator      operator_executer::add_and_run        operator_executer.cc:19-26
 *                             with the operator classes of           operator.hpp:64-1324
 *   gs_plan_run_pipeline      token_test.cc test_spmm_* functions    token_test.cc:1003-1582
 *   gs_set_config_int         set_config                              config.cc:17-40
 *   gs_get_config_int         get_config                              config.cc:42-70
 *   gs_plan_compile           code_generator::compile                code_generator.hpp:265-269
 *   gs_plan_generate_program  code_generator::generate_final_program code_generator.hpp:271-280
 *   gs_plan_upload / gs_spmm  the generated program's device copies + kernel launch
 *                             (code_generator.cc:285-600, executor.cc:6-104)
 *   gs_plan_array_*           meta_data_set::get_element / output_format_to_dir (plan arrays by key)
 *   gs_plan_from_mtx          the one-call form proposed in SURVEY.md §8b
 */
#ifndef GENERALSPARSE_H
#define GENERALSPARSE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct gs_plan gs_plan_t;
typedef void *gs_stream_t; /* hipStream_t; NULL = default stream */

enum { GS_OK = 0, GS_ERR = -1, GS_ERR_ARG = -2, GS_ERR_HIP = -3,
       GS_ERR_DEVICE = -4 /* a kernel reported a fault in its device error word (gs_plan_device_status) */ };
enum { GS_F32 = 0, GS_F16 = 1 };

typedef struct {
    const char *pipeline;   /* token_test pipeline name, see gs_plan_run_pipeline */
    int dtype;              /* GS_F32 / GS_F16 (A values, B and C) */
    int dense_n;            /* DENSE_MATRIX_SIZE used to size the plan (token_test argv[2]) */
    int p0, p1;             /* pipeline parameters (sparse_coarsen_factor / rows per BMTB / ...) */
    int ones_values;        /* 1: reference reader semantics, every value := 1 (struct.cc:186-200) */
    int device;             /* HIP device ordinal */
} gs_opts;

typedef struct {
    uint64_t rows, cols, nnz;     /* original matrix */
    uint64_t nnz_stored;          /* after padding */
    uint64_t n_units;             /* BMTs / BMWs / BMTBs the kernel walks */
    uint64_t device_bytes_A;      /* HBM bytes of A (metadata + cols + vals) per replica */
    int family;                   /* 1 thread_total, 2 warp_rows, 3 block_rows, 4 bitmap_segment */
    int col_bytes, dtype, replicas, needs_memset;
    char kernel_name[64];
    /* row-block kernels built at upload for dense width lds_n: 1 = LDS-stationary B
     * (k_lds_rows, config LDS_STAGE_B), 2 = matrix cores (k_mfma_rows, MFMA_TILES),
     * 3 = 2:4 panels of a col-direction plan on the sparse matrix cores (k_nm_mfma, NM_MFMA) */
    int lds_stage;
    uint32_t lds_n, lds_kc, lds_chunks, lds_waves;
    uint64_t lds_bytes, tile_bytes;
    uint32_t ksplit;              /* k_mfma_rows workgroups per row block (K ranges, fp32 slab combine) */
    int n_kernels;                /* kernels gs_spmm runs: 1, or one per sub-matrix of a row division */
    char device_kernel[32];       /* the device kernel gs_spmm launches at the plan's N (first sub-matrix) */
    int index_formulas;           /* index arrays the kernel evaluates as formulas (MODEL_DRIVEN_COMPRESS) */
    uint64_t index_bytes_saved;   /* u32 index bytes per replica those formulas keep out of HBM */
    uint32_t ks_nt;               /* k_mfma_ks: A's groups by non-temporal loads (KS_NT) */
    uint32_t ks_head_groups;      /* k_mfma_ks: groups per head step (KS_HEAD; 0: every step by record) */
    uint32_t nm_tiles;            /* k_nm_mfma: 16-row tiles per workgroup (NM_TILES / the upload's rule) */
} gs_plan_info;

const char *gs_last_error(void);
const char *gs_version(void);

void gs_opts_default(gs_opts *o);

/* Both readers refuse (GS_ERR -1, gs_last_error names the cause) a matrix without entries
 * (struct.cc:258), rows out of order (struct.cc:120-131), a .mtx index that is not a decimal
 * >= 1, and any index past 2^32 - 2 (dims at most 2^32 - 1); the dims grow to the largest index + 1.  row / col / val hold
 * nnz entries each (val may be NULL: every value 1). */
int gs_plan_create_from_mtx(const char *path, int ones_values, gs_plan_t **out);
int gs_plan_create_from_coo(uint64_t n_rows, uint64_t n_cols, uint64_t nnz, const uint64_t *row,
                            const uint64_t *col, const float *val, gs_plan_t **out);
int gs_set_config_int(const char *key, long long value);
/* the current value of an integer / bool key (the reference reads get_config per use,
 * config.cc:42-70) */
int gs_get_config_int(const char *key, long long *value);

/* operator surface: name = reference class name; args in constructor order
 * without the code_generator / operator_context arguments */
int gs_plan_add_operator(gs_plan_t *p, const char *op_name, const long long *args, int nargs);
/* canned pipelines: thread_total(p0=sparse_cf,p1=cf), warp_total(cf=p1), block_total(p0=rows per BMTB, cf=p1),
 * thread_bit_map(p0=sparse_cf,p1=cf), warp_segment(p0=sparse_cf,p1=cf),
 * tblock_warp_total(p0=rows per BMTB, p1=rows per BMW), balanced_warp_total(p0=nnz per BMW) */
int gs_plan_run_pipeline(gs_plan_t *p, const char *name, int dense_n, int p0, int p1);
/* sub-matrices (§8f rank 3): after fixed_interval_row_matrix_div_operator
 * (operator/fixed_interval_row_matrix_div_operator.cc:85-150; new sub-matrix ids = max + 1,
 * one per non-empty row interval) each sub-matrix gets its own operators / pipeline --
 * the reference's code_generator(meta, sub) per sub-matrix (code_generator.cc:14-40).
 * Compile / upload / gs_spmm then cover every live sub-matrix, one kernel each, in id
 * order on the caller's stream (rows of empty intervals are zeroed first). */
int gs_plan_add_operator_sub(gs_plan_t *p, int sub, const char *op_name, const long long *args, int nargs);
int gs_plan_run_pipeline_sub(gs_plan_t *p, int sub, const char *name, int dense_n, int p0, int p1);
/* ids of the sub-matrices holding nonzeros (ascending); returns the count (< 0: error) */
int gs_plan_sub_matrices(gs_plan_t *p, int *ids, int cap);
int gs_plan_compile(gs_plan_t *p);
int gs_plan_generate_program(gs_plan_t *p, const char *root_dir, int repeat, char *dir_out, int dir_out_len);

int gs_plan_upload(gs_plan_t *p, int dtype, int device);
int gs_plan_add_replica(gs_plan_t *p);
/* C = A * B.  B: K x N row-major, C: M x N row-major, device pointers of the
 * plan's dtype.  Enqueued on `stream`; returns without synchronising.  The library cannot
 * see the extents behind raw pointers: the caller guarantees K x N readable and M x N
 * writable elements (the Python Plan.spmm / Rotation / Batch check their tensors). */
int gs_spmm(gs_plan_t *p, const void *B, void *C, int N, gs_stream_t stream);
int gs_spmm_replica(gs_plan_t *p, int replica, const void *B, void *C, int N, gs_stream_t stream);
/* `count` SpMMs enqueued back to back from native code, call i using replica
 * (first + i) % replicas with B_ptrs / C_ptrs entry (first + i) % n_ptrs
 * (bench rotation without a host round trip per launch) */
int gs_spmm_rotate(gs_plan_t *p, int count, int first, const void *const *B_ptrs, void *const *C_ptrs, int n_ptrs,
                   int N, gs_stream_t stream);
/* n SpMMs (plans[i], replicas[i], B[i], C[i]) enqueued on `stream` in order: a batch of
 * independent matrices (a layer's weights).  Replaces the reference's one launch per
 * sub-matrix in its multi-kernel executor (operator_executer.hpp:62-76, executor.cc:6-104):
 * consecutive entries whose plans run the K-split matrix-core kernel at N = 32 with one
 * instantiation (up to 32 of them, each a distinct (plan, replica)) are ONE grouped launch
 * (k_mfma_ks_group); the others launch as gs_spmm_replica does. */
int gs_spmm_batch(gs_plan_t *const *plans, const int *replicas, const void *const *B, void *const *C, int n, int N,
                  gs_stream_t stream);

/* how gs_spmm_batch would enqueue the batch: returns the number of launches (< 0: error) and
 * the entries each launch carries in entries_per_launch[0 .. min(count, cap)) (a grouped
 * k_mfma_ks_group launch carries up to 32) */
int gs_batch_launches(gs_plan_t *const *plans, const int *replicas, int n, int N, int *entries_per_launch, int cap);
/* synchronises the device (every stream: launches of the plan on side streams must have
 * ended before the words are read and cleared; `stream` is kept for the signature) and reads
 * the plan's device error words (every replica, every
 * sub-matrix kernel): GS_ERR_DEVICE when a launch reported a fault since the last call --
 * a K-split combine that gave up waiting for a partial slab (its rows of C are NaN) --
 * 0 otherwise.  The words are cleared once reported.  The reference asserts on the host
 * after its kernels (executor.cc:6-104 checks cudaGetLastError); this is the device side. */
int gs_plan_device_status(gs_plan_t *p, gs_stream_t stream);

int gs_plan_info_get(gs_plan_t *p, gs_plan_info *info);
int gs_plan_array_count(gs_plan_t *p);
int gs_plan_array_key(gs_plan_t *p, int i, char *buf, int buf_len);
long long gs_plan_array_len(gs_plan_t *p, const char *key);      /* -1 if absent */
int gs_plan_array_is_float(gs_plan_t *p, const char *key);
int gs_plan_array_read_u64(gs_plan_t *p, const char *key, uint64_t *out, uint64_t n);
int gs_plan_array_read_f64(gs_plan_t *p, const char *key, double *out, uint64_t n);
int gs_plan_log(gs_plan_t *p, char *buf, int buf_len); /* operator / transform history */

/* model-driven index compression of one integer plan array (code_generator.cc:2618-3063,
 * the if_*_compress / get_*_compress pairs; honours MODEL_DRIVEN_COMPRESS): kind_out gets
 * "none" | "linear" | "branch" | "cycle_linear" | "cycle_increase" | "residual", expr_out the
 * expression of `idx` the generated kernel evaluates; *exact = 1 when the formula reproduces
 * the array (the reference's acceptance tests admit some it does not).  A residual adds
 * "<POS>_<name>_res_<sub>" to the plan. */
int gs_plan_index_compression(gs_plan_t *p, const char *key, char *kind_out, int kind_len, char *expr_out,
                              int expr_len, int *exact);
/* the same analysis of a raw array (type_ori: the gs data_type code of its storage type) */
int gs_index_compression_of_array(const uint64_t *a, uint64_t n, int type_ori, int branch_max, char *kind_out,
                                  int kind_len, uint64_t *params /* coef, intercept, cycle, aa, bb */, int *exact);

/* diagnostics (not part of the reference surface): one launch of the matrix-core
 * kernel's timestamped build; stamps[g*64 + i] = s_memtime of phase i in workgroup g
 * (0 start, 1 loads issued, 2 first barrier, 3 first chunk staged, 4+5j.. per chunk j:
 * top barrier, loads+clear issued, MFMA done, mid barrier, next chunk staged; 63 end) */
int gs_debug_mfma_timeline(gs_plan_t *p, const void *B, void *C, int N, gs_stream_t stream, uint64_t *stamps,
                           uint64_t n_stamps);

/* binary plan files: a compiled plan (kernel selection + every plan
 * array) in one file, loaded without re-running the transforms; upload before gs_spmm */
int gs_plan_save(gs_plan_t *p, const char *path);
int gs_plan_load(const char *path, gs_plan_t **out);

/* logical_check (metadata_set.cc:806-1890): cross-array consistency of the plan's metadata
 * (the reference's checks, with its relative-vs-absolute checks made exact); 0 consistent,
 * 1 a violation (described in msg), < 0 error.  gs_plan_compile runs it and fails on a
 * violation, as token_test asserts it after every pipeline. */
int gs_plan_logical_check(gs_plan_t *p, char *msg, int msg_len);
/* metadata editing (tools and tests): entry i of an integer plan array */
int gs_plan_array_set_u64(gs_plan_t *p, const char *key, uint64_t i, uint64_t value);

/* one call: read + pipeline + compile + upload */
int gs_plan_from_mtx(const char *path, const gs_opts *opts, gs_plan_t **out);
void gs_plan_free(gs_plan_t *p);

#ifdef __cplusplus
}
#endif
#endif
