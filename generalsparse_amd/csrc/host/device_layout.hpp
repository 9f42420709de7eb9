// host/device_layout.hpp -- the HBM layouts of the matrix-core kernels (k_mfma_rows,
// k_mfma_ks, k_nm_mfma), built on the host from a compiled plan.  Shared by the device
// upload (kernels/device_plan.hip) and the code generator (code_generator.cc), so the
// program generate_final_program emits launches exactly the layout gs_spmm runs.
#pragma once

#include "gs_core.hpp"
#include "code_generator.hpp"
#include "../hip_code/kernel_consts.hpp"

#include <string>
#include <vector>

namespace gs {

constexpr uint32_t kMfmaThreads = 64 * gsk::kMfmaWaves;
// k_mfma_ks workgroup waves, entry sets in flight per wave (look-ahead D: 2 measured fastest
// over C2 and the OPT-30B shapes -- 1-12% under D = 4, D = 1 / 3 / 6 slower, profiles/r04o_*)
constexpr uint32_t kKsWaves = 8, kKsDepth = 2;

// fp32 -> fp16 bits, round to nearest even (bit-identical to the device conversion)
uint16_t f32_to_f16_bits(float f);

struct canon_rows {
    std::vector<uint32_t> rp;
    std::vector<uint64_t> col;
    std::vector<float> val;
};

canon_rows canonical_rows(const std::vector<uint32_t> &rp, const std::vector<uint64_t> &col, const universal_array &vals);

// k_mfma_rows upload layout (kernel_lib.hpp): per (BMTB g, 2^lgKC-column chunk j), the
// chunk's entries in groups of 8 = [8 x u16 halfword position in the dense image] +
// [8 x f16]; seg_start[g*nc + j] the first group
struct mfma_tiles {
    uint32_t lgKC = 0, nc = 0, RT = 0, RMAX = 0, MAXA = 0, gmax = 0;
    size_t lds_bytes = 0;
    std::vector<uint32_t> seg_start;  // in groups
    std::vector<uint16_t> pos, val;   // 8 u16 per group each, + one spare group
};

size_t mfma_lds_bytes(uint32_t lgKC, uint32_t CT, uint32_t RMAX);
// LDS one k_mfma_rows variant needs (B ring + dense images, or the compute waves' partial tiles)
size_t mfma_rows_lds_need(uint32_t lgKC, uint32_t CT, uint32_t RT, uint32_t RMAX, int glds, int nbg, int wct);
bool build_mfma_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                      const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                      size_t lds_budget, int64_t max_fill, mfma_tiles &t, std::string &why);

// k_mfma_ks upload layout (device_layout.cc build_ks_tiles): the groups of every (BMTB g,
// K range q, 32-column k-step s) back to back in (unit u = g*S + q, s) order, located by
// steps[2*(u*NS + s)] = first group and steps[2*(u*NS + s) + 1] = group count (at most
// GCAP, the plan's largest step: it sets MAXG), + one spare group
struct ks_tiles {
    uint32_t S = 0, NS = 0, RT = 0, RMAX = 0, MAXG = 0, GCAP = 0, W = 0;
    uint32_t CT = 0;  // 16-column MFMA tiles per workgroup (ks_ct_rt)
    bool AP = true;   // partial tiles beside the stages (ks_red_apart; KS_APART)
    bool P8 = false;  // 8-bit positions (KS_POS8): pos8 instead of pos, see build_ks_tiles
    uint32_t NT = 0;  // k_mfma_ks NTL: 1 = A's groups by non-temporal loads (KS_NT; N = 32, 8 waves, apart layout)
    // head steps (KS_HEAD): the first W x kKsDepth k-steps of every unit -- the ones each wave loads
    // in its prologue -- have their groups at a fixed place, (unit * HS + step) * GH with HS =
    // min(W * kKsDepth, NS), padded with
    // zero-row groups to GH groups, so the prologue's group loads need no record round trip; their
    // records still describe them (first group, count), so a kernel may also take them by record
    uint32_t GH = 0;  // groups per head step (0: no head region)
    size_t lds_bytes = 0;
    std::vector<uint16_t> pos, val;  // 8 u16 per group each
    std::vector<uint8_t> pos8;       // P8: 8 bytes per group
    std::vector<uint32_t> steps;     // per (unit, k-step): first group, group count
};

// k_mfma_ks column tiles: CT 16-column MFMA tiles per workgroup (N = 8 runs one partial
// tile), ks_col_tiles(N) tiles in the grid's y dimension (N = 128: two)
inline uint32_t ks_ct(uint32_t N) { return N <= 16 ? 1u : (N <= 32 ? 2u : 4u); }
inline uint32_t ks_col_tiles(uint32_t N) { return (N + 16 * ks_ct(N) - 1) / (16 * ks_ct(N)); }
// k_mfma_ks's own choice: N >= 128 with row blocks of at most 48 rows (RT <= 3) runs 128 columns
// per workgroup (CT = 8: 96 fp32 accumulators, 255 VGPRs, no spill), so A is read once at N = 128
// instead of once per 64-column tile; taller blocks keep CT = 4 (their accumulators would spill)
inline uint32_t ks_ct_rt(uint32_t N, uint32_t RT) { return N >= 128 && RT <= 3 ? 8u : ks_ct(N); }
// ... and the 128-column instantiations that hold their registers (no spill): 32-row blocks with up to
// 192 entry groups per k-step, 48-row blocks with up to 64; other plans at N >= 128 take CT = 4
inline bool ks_ct8_fits(uint32_t RT, uint32_t MAXG) { return (RT == 2 && MAXG <= 3) || (RT == 3 && MAXG == 1); }
inline uint32_t ks_col_tiles_ct(uint32_t N, uint32_t CT) { return (N + 16 * CT - 1) / (16 * CT); }

bool build_ks_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                    const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                    int64_t s_cfg, int64_t min_rows, int64_t max_fill, ks_tiles &t, std::string &why);

// k_mfma_bm upload layout: unit u = (BMTB g, K range q) of NS 32-column k-steps; per
// (u*NS + step)*64 + lane one 8-byte record (rec[2i] = mask bytes of tiles 0..3, rec[2i+1]
// = tiles 4..5 | u16 value offset << 16), sbase[u*NS + step] the step's first value, the
// values (f16 bits) lane after lane, tile after tile, ascending columns (+ 16 halves pad)
struct bm_tiles {
    uint32_t S = 0, NS = 0, RT = 0, RMAX = 0, W = 0;
    bool kb = false;  // k_mfma_kb (8 waves, k_mfma_ks pipeline)
    uint32_t NVB = 0;  // ... KB of values per k-step (1, 2 or 4)
    bool v2 = false;  // k_mfma_bm2 (one wave per row tile, B slice resident in LDS)
    size_t lds_bytes = 0;
    std::vector<uint32_t> rec;
    std::vector<uint32_t> sbase;
    std::vector<uint16_t> val;
};

bool build_bm_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                    const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                    int64_t s_cfg, int64_t waves, int64_t max_fill, bm_tiles &t, std::string &why);

// k_nm_mfma upload layout: one 4,608-B block per (64-row group, 64-column k-step)
bool build_nm_panels(const std::vector<uint64_t> &rows, const std::vector<uint64_t> &col, const universal_array &vals,
                     uint64_t row_num, uint64_t K, std::vector<unsigned char> &blk, uint32_t &S, std::string &why,
                     uint32_t T = 8);
// k_nm_mfma's 16-row tiles per workgroup for a row count (NM_TILES = 0): among T = 8, 7, 4, 2
// (7 only below N = 128) the fewest tiles per CU (ceil(workgroups / 256 CUs) x T), ties to the
// larger T
uint32_t nm_tiles_for(uint64_t row_num, int64_t cfg_tiles, uint32_t N);

// The matrix-core layout gs_spmm runs for a compiled plan at its dense width
// (DENSE_MATRIX_SIZE), chosen and built once here for both the device upload and the
// emitted program: k_nm_mfma for col-direction 2:4 panels, k_mfma_ks for row blocks of
// >= KS_MIN_ROWS rows, k_mfma_rows for the other fp16 BMTB plans; NONE = a gather family.
// The k_mfma_rows variant (B by LDS-DMA or registers, ring depth, compute waves) is fixed
// here from the config, so the LDS size and the launch agree whatever changes later.
struct mc_layout {
    enum kind_t { NONE, ROWS, KS, NM, BM } kind = NONE;
    uint32_t N = 0;
    std::vector<uint64_t> tbr;  // BMTB first rows (ROWS, KS)
    mfma_tiles rows;
    uint32_t rows_ksplit = 1, rows_ncs = 0;  // k_mfma_rows K ranges per row block, chunks per range
    int rows_glds = 2, rows_nbg = 3, rows_wct = 6, rows_maxa = 1;  // k_mfma_rows template arguments
    bool rows_flags = false;  // ... FLG (MFMA_FLAGS: LDS counter hand-offs, GLDS 2 / NBG 3 / 6 compute waves)
    ks_tiles ks;
    bm_tiles bm;
    std::vector<unsigned char> nm_blk;  // k_nm_mfma blocks
    uint32_t nm_S = 0;                  // ... k-steps per row group
    uint32_t nm_T = 8;                  // ... 16-row tiles per workgroup (nm_tiles_for)
    uint64_t nm_rows = 0;
    bool nm_ks = false;                    // k_nm_mfma_ks (256-row workgroups, K split) instead of k_nm_mfma
    bool nm4 = false;                      // k_nm_mfma4 (256-row workgroups of 8 waves, K split, B by LDS-DMA)
    bool nm_nt = false;                    // k_nm_mfma: A's panel blocks by non-temporal loads (NM_NT)
    uint32_t nm_split = 1, nm_ncs = 0;     // ... K ranges per row block, 256-column chunks per range
    std::string why;  // why NONE
};
mc_layout choose_matrix_core_layout(const meta_data_set &m, const kernel_spec &sp, int sb, uint64_t K, int dtype);

}  // namespace gs
