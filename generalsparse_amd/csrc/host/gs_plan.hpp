// gs_plan.hpp -- internal state behind the C ABI handle gs_plan_t.
#pragma once

#include "operator.hpp"
#include "device_layout.hpp"
#include "../hip_code/idx_formula.hpp"

#include <hip/hip_runtime.h>

namespace gs {

// Device copies of the arrays one kernel family consumes, in the layout the
// gfx950 kernels want (narrowest index types, A streams padded so aligned
// over-reads stay in bounds).  One replica = one independent copy of A
// (bench.py rotates replicas past the 256 MB Infinity Cache).
struct device_arrays {
    void *col = nullptr, *val = nullptr;
    void *pad_out = nullptr;  // row-padded plans: scratch output of all the plan's rows
    void *tcol = nullptr, *tval = nullptr;  // LDS tile layout (k_lds_rows)
    uint32_t *t0 = nullptr, *t1 = nullptr, *t2 = nullptr, *t3 = nullptr, *t4 = nullptr;
    uint32_t *a0 = nullptr, *a1 = nullptr, *a2 = nullptr, *a3 = nullptr, *a4 = nullptr;
    uint64_t *m0 = nullptr;
    float *ws = nullptr;  // k_mfma_rows K-split slabs (per replica: a replica never runs concurrently with itself)
    float *ws2 = nullptr;  // k_merge_path: partials of the rows each wave closes first (head_rec)
    uint32_t *cperm = nullptr;  // merge path, MP_COL_PERM: original column of each renumbered column (or, with
                                // perm_scatter, the new place of each column)
    void *bperm = nullptr;      // ... B gathered into that order (K x the plan's N, per replica)
    // merge path, MP_COL_PARTS: kMpPartPtrs device arrays per column partition (mp_part_* below)
    std::vector<void *> pp;
};
// per column partition x: pp[x * kMpPartPtrs + i], i = the mp_part_* index
enum { MP_PART_COL, MP_PART_VAL, MP_PART_WZ, MP_PART_WQ, MP_PART_ENDS, MP_PART_RID, MP_PART_EMPTY, MP_PART_WS,
       MP_PART_WS2, MP_PART_T0, MP_PART_CHAIN, MP_PART_CNT, MP_PART_OUT, kMpPartPtrs };

struct device_plan {
    int device = 0;
    int dtype = 1;         // 0 fp32, 1 fp16 (values, B and C)
    int col_bytes = 2;     // 2 (u16) or 4 (u32)
    int scf = 4;           // sparse entries per vector load
    bool needs_memset = false;
    uint64_t n_out_rows = 0;  // one past the last row of C this plan writes
    uint64_t pad_rows = 0;    // row-padded plan (modify_*_by_row_pad_in_sub_matrix): its rows, > M
    uint32_t pad_N = 0;       // ... the dense width its scratch output holds
    uint64_t out_lo = 0;      // first row of C this plan writes (a sub-matrix's range)
    uint64_t n_units = 0;     // BMTs / BMWs / BMTBs the grid walks
    uint64_t n_rows_aux = 0;  // rows covered (thread_total: rows incl. trailing empty)
    uint64_t row_base = 0;
    uint32_t ks_ctw = 0;      // k_mfma_ks: 16-column tiles per workgroup (ks_tiles::CT)
    bool ks_ap = true;        // k_mfma_ks: partial tiles beside the stages (ks_tiles::AP)
    bool ks_p8 = false;       // k_mfma_ks: 8-bit entry positions (ks_tiles::P8, KS_POS8)
    uint32_t ks_gh = 0;       // k_mfma_ks: groups per head step (ks_tiles::GH; 0: every step by record)
    uint32_t ks_nt = 0;       // k_mfma_ks: non-temporal loads of A's groups (NTL bit 0; ks_tiles::NT, KS_NT)
    uint32_t ks_persist = 0;  // k_mfma_ks: persistent grid of this many workgroups pulling units (KS_PERSIST, experiments)
    bool nm_nt = false;       // k_nm_mfma: non-temporal panel loads (NM_NT)
    uint32_t nm_tiles = 8;    // k_nm_mfma: 16-row tiles per workgroup (mc_layout::nm_T)
    bool lds_dma = false;     // k_lds_rows_dma: fp32 N = 32 chunks by LDS-DMA into two buffers (LDS_DMA)
    // merge path, MP_COL_PARTS: the columns (renumbered by degree, MP_COL_PERM) dealt round-robin
    // over mp_parts partitions; one k_merge_path per partition, each over its own CSR and wave
    // ranges, so every pass gathers B rows of one partition only (its hubs fit each XCD's L2)
    uint32_t mp_parts = 0;
    std::vector<uint32_t> mp_part_W, mp_part_rows, mp_part_fin;
    uint64_t err_at = 0;      // K-split combine: index of the device error word in t2 (0: none)
    uint64_t nnz_stored = 0;  // padded nnz on device
    size_t bytes_A = 0;       // device bytes of A per replica (metadata + cols + vals)
    // LDS-stationary B (k_lds_rows): chunk geometry fixed for dense width lds_N
    bool lds = false;
    bool nm_ks = false;  // k_nm_mfma_ks (ksplit K ranges of ncs chunks; ws slabs + t2 counters when ksplit > 1)
    bool nm = false;    // k_nm_mfma: 2:4 panels of a col-direction plan (A blocks in tcol; k-steps in KC)
    bool nm4 = false;   // ... on k_nm_mfma4 (256-row workgroups, ksplit K ranges of ncs chunks)
    bool mfma = false;  // k_mfma_rows (uses KC, nc, lds_bytes; log2 KC in RSB; RT in maxr; RMAX in rpw_max)
    bool ks = false;    // k_mfma_ks: K split over ksplit workgroups per row block, B slice in LDS
                        // (t0 BMTB rows, tcol/tval groups; ks_ns k-steps per range,
                        // RT in maxr, MAXG in seg_cap, ws slabs + t2 arrivals when ksplit > 1)
    uint32_t ks_ns = 0, ks_gcap = 0;
    bool bmkb = false;  // ... k_mfma_kb: k_mfma_ks pipeline on the bitmap layout (8 waves)
    bool bm2 = false;   // ... k_mfma_bm2: one wave per row tile (W = RT), B slice of ks_ns k-steps in LDS
    bool bm = false;    // k_mfma_bm: bitmap records (tcol), step bases (t1), values (tval), t0 BMTB rows;
                        // ksplit K ranges of ks_ns k-steps, RT in maxr, W in waves

    bool mp_rows = false;   // merge-path plans: k_merge_rows (fixed at upload, MP_ROWS), else k_merge_path
    uint32_t mp_solo = 16;
    bool col_perm = false;  // merge path: columns renumbered by degree (cperm / bperm)
    bool perm_scatter = false;  // ... cperm holds each column's new place (k_permute_rows scatters)  // k_merge_rows: slot-alone row length (MP_SOLO)
    // k_mfma_rows variant fixed at upload (device_layout.cc): GLDS / B ring depth / compute
    // waves / entry groups per thread -- the launch uses these, not the config of the moment
    int mfma_glds = 2, mfma_nbg = 3, mfma_wct = 6, mfma_maxa = 1;
    bool mfma_flags = false;  // k_mfma_rows: LDS counter hand-offs instead of per-chunk barriers  // k_mfma_ks: k-steps per K range, entry groups per step
    std::string kernel;  // the device kernel gs_spmm launches at the plan's N (empty: the family's)
    uint32_t ksplit = 1, ncs = 0;  // k_mfma_rows workgroups per row block, chunks per workgroup
    uint32_t ws_n = 0;             // bitmap family: dense width of the fp32 workspace
    uint64_t n_fin = 0;            // bitmap family: rows k_finalize_rows writes
    uint32_t span = 0;             // k_row_chunks: BMTs per wave
    uint32_t bmw_rows_max = 0;     // k_warp_rows: most rows in one BMW
    double mean_row_nnz = 0.0;     // ... and the mean row length (slots per row)
    uint32_t ilv = 0;              // k_row_chunks: BMT size of an interleaved layout (0: contiguous)
    uint32_t lds_N = 0, KC = 0, nc = 0, RSB = 0, rpw_max = 0, seg_cap = 0, waves = 0, maxr = 0;
    size_t lds_bytes = 0, bytes_tile = 0;
    // model-driven index compression on the device (MODEL_DRIVEN_COMPRESS):
    // the formulas the gather families evaluate for a0 / a1 (kind IDX_ARRAY: read the array)
    gsk::idx_formula f0, f1;
    int index_formulas = 0;         // arrays replaced by a formula (or narrowed to residuals)
    uint64_t index_bytes_saved = 0;  // u32 index bytes per replica not uploaded because of them
    std::vector<device_arrays> replicas;
    std::vector<void *> allocations;  // everything to hipFree
};

struct plan_state {
    std::shared_ptr<meta_data_set> meta;
    std::shared_ptr<code_generator> cg;
    std::shared_ptr<operator_executer> exec;
    std::string pipeline;
    uint64_t M = 0, K = 0, nnz = 0;
    device_plan dev;
    bool uploaded = false;
    // a sub-matrix of row_nz_matrix_div_operator: its row indices refer to the divided
    // sub-matrix (rows [parent_row_base, parent_row_base + parent_rows) of C); -1 otherwise
    int64_t parent_row_base = -1;
    uint64_t parent_rows = 0;
};

// a kernel of a plan file: sub-matrix id, kernel spec, parent-indexed row range
struct loaded_kernel {
    int sub = 0;
    kernel_spec spec;
    int64_t parent_row_base = -1;
    uint64_t parent_rows = 0;
};

// plan_io.cc: binary plan files
// one file holds every kernel of a plan (one per sub-matrix of a row division); load
// returns the metadata set and the (sub-matrix id, kernel spec) list
void save_plan(const std::vector<const plan_state *> &kernels, const std::string &path);
std::shared_ptr<meta_data_set> load_plan(const std::string &path, std::vector<loaded_kernel> &kernels,
                                         std::string &pipeline);

// device_plan.hip
void upload_plan(plan_state &p, int dtype, int device);
void add_replica(plan_state &p);
void free_device(plan_state &p);
// zero rows [lo, hi) of a row-major C of width N, element size e (sub-matrix executor)
void memset_rows(void *C, uint64_t lo, uint64_t hi, uint32_t N, size_t e, hipStream_t stream);
// C[row0 + r] = sum of parts[q][r] over the q with r < rows[q], r < P (parent-indexed
// sub-matrices' scratch outputs; parts / rows are device arrays of n entries)
void combine_parts(const void *const *parts, const uint32_t *rows, uint32_t n, void *C, uint64_t row0, uint64_t P,
                   uint32_t N, int dtype, hipStream_t stream);
void launch_spmm(plan_state &p, int replica, const void *B, void *C, uint32_t N, hipStream_t stream);
// uploads the CSR arrays a matrix-core plan deferred (every replica), for a launch at another dense width
void ensure_csr(plan_state &p);
void debug_mp_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host);
void debug_mfma_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                         size_t n_host);
// mfma_launch.hip: k_mfma_rows / k_nm_mfma (and k_mfma_ks through launch_ks) at the plan's N
void launch_mfma(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s);
void launch_nm(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s);
// gather_launch.hip: the CUDA-core gather families and k_lds_rows
void launch_gather(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s);
// ks_launch.hip: k_mfma_ks (K-split, wave-autonomous matrix-core row blocks)
void launch_ks(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s);
// grouped k_mfma_ks launches (gs_spmm_batch): one grid over up to 32 entries of one
// instantiation (equal nonzero ks_group_key); every entry a distinct (plan, replica)
struct ks_group_item {
    const plan_state *p;
    int replica;
    const void *B;
    void *C;
};
uint32_t ks_group_key(const plan_state &p, uint32_t N);  // 0: not groupable
void launch_ks_group(const std::vector<ks_group_item> &it, uint32_t N, hipStream_t s);
void launch_bm(const plan_state &p, const device_arrays &a, const void *B, void *C, uint32_t N, hipStream_t s);
void debug_bm_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host);
void debug_ks_timeline(const plan_state &p, const void *B, void *C, uint32_t N, hipStream_t s, uint64_t *host,
                       size_t n_host);

}  // namespace gs
