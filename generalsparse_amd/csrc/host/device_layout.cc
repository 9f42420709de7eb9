// host/device_layout.cc -- matrix-core HBM layouts (see device_layout.hpp).
#include "device_layout.hpp"

#include <algorithm>
#include <cstring>

namespace gs {

uint16_t f32_to_f16_bits(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    const uint32_t sign = (x >> 16) & 0x8000u, exp = (x >> 23) & 0xffu;
    uint32_t man = x & 0x7fffffu;
    if (exp == 0xffu) return (uint16_t)(sign | 0x7c00u | (man ? (0x200u | (man >> 13)) : 0u));  // inf, quiet nan
    const int e = (int)exp - 127 + 15;
    if (e >= 31) return (uint16_t)(sign | 0x7c00u);  // overflow: inf
    if (e <= 0) {                                    // fp16 subnormal or zero
        if (e < -10) return (uint16_t)sign;
        man |= 0x800000u;
        const int shift = 14 - e;
        uint32_t hm = man >> shift;
        const uint32_t rem = man & ((1u << shift) - 1u), halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (hm & 1u))) hm++;
        return (uint16_t)(sign | hm);
    }
    uint32_t h = sign | ((uint32_t)e << 10) | (man >> 13);
    const uint32_t rem = man & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;  // a carry into the exponent is right
    return (uint16_t)h;
}

// Rows as the matrix-core layouts need them: each row's columns ascending and
// distinct.  The reference accepts any column order inside a row and its gather
// kernels add repeated coordinates, so entries are stably sorted by column and
// repeated ones summed (in double, rounded to fp32 once).  rp is the CSR row
// pointer of the plan's (row-sorted) COO.


canon_rows canonical_rows(const std::vector<uint32_t> &rp, const std::vector<uint64_t> &col, const universal_array &vals) {
    canon_rows c;
    const uint64_t nr = rp.size() - 1;
    c.rp.assign(nr + 1, 0);
    c.col.reserve(col.size());
    c.val.reserve(col.size());
    std::vector<std::pair<uint64_t, uint64_t>> ent;  // (col, position)
    for (uint64_t r = 0; r < nr; r++) {
        bool ordered = true;
        for (uint64_t e = rp[r] + 1; e < rp[r + 1]; e++) ordered &= col[e] > col[e - 1];
        if (ordered) {
            for (uint64_t e = rp[r]; e < rp[r + 1]; e++) {
                c.col.push_back(col[e]);
                c.val.push_back((float)vals.read_float_from_arr(e));
            }
        } else {
            ent.clear();
            for (uint64_t e = rp[r]; e < rp[r + 1]; e++) ent.push_back({col[e], e});
            std::stable_sort(ent.begin(), ent.end(), [](const auto &a, const auto &b) { return a.first < b.first; });
            for (size_t i = 0; i < ent.size();) {
                double sum = 0;
                size_t j = i;
                for (; j < ent.size() && ent[j].first == ent[i].first; j++) sum += vals.read_float_from_arr(ent[j].second);
                c.col.push_back(ent[i].first);
                c.val.push_back((float)sum);
                i = j;
            }
        }
        GS_CHECK(c.col.size() < 0xffffffffull, "nnz exceeds 32-bit offsets");
        c.rp[r + 1] = (uint32_t)c.col.size();
    }
    return c;
}

// ------------------------------------------------------------------ MFMA tiles
// Upload layout of k_mfma_rows (kernel_lib.hpp): for BMTB g and column chunk j,
// the entries of g's rows with columns in [j*KC, (j+1)*KC), in groups of 8:
// pos[] = 8 x u16 halfword index in the dense image (local_row*(KC+16) +
// local_col), val[] = 8 x f16; the last group is padded with (row R, value 0),
// row R being the kernel's zero row.


constexpr uint32_t kMfmaBThreads = 64 * gsk::kMfmaBWaves, kMfmaAThreads = 64 * gsk::kMfmaAWaves;

size_t mfma_lds_bytes(uint32_t lgKC, uint32_t CT, uint32_t RMAX) {
    const size_t KC = 1ull << lgKC;
    // the larger of the two layouts (2 B buffers + 3 dense images; MFMA_GLDS: MFMA_GLDS_NBUF + 2)
    const size_t nb = (size_t)std::max<int64_t>(3, get_config().MFMA_GLDS_NBUF);
    const size_t szB = KC * 32 * CT, szD = (RMAX + 1) * (2 * KC + 32);
    return std::max(2 * szB + 3 * szD, nb * szB + 2 * szD) + 1024;  // + stamp slots and the arrival flag
}

size_t mfma_rows_lds_need(uint32_t lgKC, uint32_t CT, uint32_t RT, uint32_t RMAX, int glds, int nbg, int wct) {
    const size_t KC = 1ull << lgKC;
    const size_t szB = KC * 32 * CT, szD = (RMAX + 1) * (2 * KC + 32);
    const size_t stage = glds ? (size_t)nbg * szB + 2 * szD : 2 * szB + 3 * szD;
    return std::max(stage, (size_t)wct * RT * CT * 1024);
}

// Order one segment's entries for the scatter: the kernel's 32-lane half-waves
// write (group q, slot e) for 32 consecutive groups at once, so every such
// "round" takes entries of distinct LDS write banks ((halfword/2) mod 32) where
// possible (greedy: fullest banks first, a bank twice only when fewer than 32
// banks remain).  Appends 8 u16 pos + 8 u16 values per group; padding slots write
// 0 into the zero row (pad_h = its first halfword), on banks of their own.
static void bank_order_segment(const std::vector<uint16_t> &pos, const std::vector<uint16_t> &val, uint32_t pad_h,
                        std::vector<uint16_t> &out_pos, std::vector<uint16_t> &out_val, uint32_t pad_slots = 32) {
    const size_t n = pos.size();
    const size_t ng = (n + 7) / 8;
    std::vector<std::vector<uint32_t>> bucket(32);
    for (uint32_t i = 0; i < n; i++) bucket[(pos[i] >> 1) & 31].push_back(i);
    const size_t base = out_pos.size();
    out_pos.resize(base + ng * 8);
    out_val.resize(base + ng * 8);
    std::vector<int> order(32);
    for (size_t b0 = 0; b0 < ng; b0 += 32) {
        const size_t gl = std::min<size_t>(32, ng - b0);
        for (int e = 0; e < 8; e++) {
            for (int k = 0; k < 32; k++) order[k] = k;
            std::stable_sort(order.begin(), order.end(),
                             [&](int a, int b) { return bucket[a].size() > bucket[b].size(); });
            size_t l = 0;
            bool progress = true;
            while (l < gl && progress) {  // one entry per bank per pass, fullest banks first
                progress = false;
                for (int k = 0; k < 32 && l < gl; k++) {
                    auto &bk = bucket[order[k]];
                    if (bk.empty()) continue;
                    const uint32_t i = bk.back();
                    bk.pop_back();
                    const size_t slot = base + (b0 + l) * 8 + e;
                    out_pos[slot] = pos[i];
                    out_val[slot] = val[i];
                    l++;
                    progress = true;
                }
            }
            for (; l < gl; l++) {  // padding: value 0 into the zero row, one bank each
                const size_t slot = base + (b0 + l) * 8 + e;
                out_pos[slot] = (uint16_t)(pad_h + 2 * (l % pad_slots));  // inside the zero row
                out_val[slot] = 0;
            }
        }
    }
    for (const auto &bk : bucket) GS_CHECK(bk.empty(), "bank ordering lost an entry");
}

// KS_POS8 layout of one k-step (k_mfma_ks with P8): the step's entries split into segments of
// 8 rows x 16 columns of the wave image -- segment sg = (row / 8) * 2 + column / 16, so row tile
// rt holds segments 4rt .. 4rt+3 -- and every group of 8 entries lies in ONE segment.  Byte e of
// a group: bit 7 = bit e of the segment id, bits 0-6 = (row % 8) << 4 | column % 16, so a group
// costs 8 + 16 bytes (3 B per nonzero against 4 B with u16 image positions).  A segment's last
// group is padded with copies of its first entry (the same value written twice to one place:
// the scatter and the clear are idempotent).  Inside a segment the entries are dealt to its
// groups so that each slot e falls on distinct LDS write banks where possible (as
// bank_order_segment).  Appends to out_pos8 / out_val; returns the groups written.
static size_t pos8_step(const std::vector<uint16_t> &row, const std::vector<uint16_t> &colw,
                        const std::vector<uint16_t> &hv, uint32_t RS, std::vector<uint8_t> &out_pos8,
                        std::vector<uint16_t> &out_val) {
    const size_t n = row.size();
    uint32_t nseg = 0;
    for (size_t i = 0; i < n; i++) nseg = std::max<uint32_t>(nseg, (uint32_t)((row[i] / 8) * 2 + colw[i] / 16) + 1);
    std::vector<std::vector<uint32_t>> seg(nseg);
    for (uint32_t i = 0; i < n; i++) seg[(row[i] / 8) * 2 + colw[i] / 16].push_back(i);
    size_t groups = 0;
    std::vector<std::vector<uint32_t>> bucket(32);
    for (uint32_t sg = 0; sg < nseg; sg++) {
        const auto &es = seg[sg];
        if (es.empty()) continue;
        GS_CHECK(sg < 256, "KS_POS8: segment id beyond 8 bits");
        const size_t ng = (es.size() + 7) / 8;
        for (auto &b : bucket) b.clear();
        for (uint32_t i : es) bucket[((uint32_t)row[i] * RS + colw[i]) / 2 % 32].push_back(i);
        std::vector<uint32_t> slot(ng * 8, UINT32_MAX);
        std::vector<int> order(32);
        for (int e = 0; e < 8; e++) {  // slot e of the segment's groups on distinct banks, fullest first
            for (int k = 0; k < 32; k++) order[k] = k;
            std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return bucket[a].size() > bucket[b].size(); });
            size_t l = 0;
            bool progress = true;
            while (l < ng && progress) {
                progress = false;
                for (int k = 0; k < 32 && l < ng; k++) {
                    auto &bk = bucket[order[k]];
                    if (bk.empty()) continue;
                    slot[l * 8 + e] = bk.back();
                    bk.pop_back();
                    l++;
                    progress = true;
                }
            }
        }
        for (const auto &bk : bucket) GS_CHECK(bk.empty(), "KS_POS8: bank ordering lost an entry");
        const uint32_t first = slot[0];
        for (size_t gi = 0; gi < ng; gi++)
            for (int e = 0; e < 8; e++) {
                const uint32_t i = slot[gi * 8 + e] == UINT32_MAX ? first : slot[gi * 8 + e];
                const uint8_t p7 = (uint8_t)(((row[i] % 8) << 4) | (colw[i] % 16));
                out_pos8.push_back((uint8_t)((((sg >> e) & 1u) << 7) | p7));
                out_val.push_back(hv[i]);
            }
        groups += ng;
    }
    return groups;
}

bool build_mfma_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                      const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                      size_t lds_budget, int64_t max_fill, mfma_tiles &t, std::string &why) {
    const uint64_t nb = tb_rows.size() - 1;
    if (nb == 0 || K == 0) { why = "empty plan"; return false; }
    if (N == 0 || N > 64 || N % 8 != 0) { why = "N must be a multiple of 8 up to 64"; return false; }
    const uint32_t CT = ks_ct(N);  // 16-column tiles (N = 8: one tile of which 8 columns are stored)
    uint64_t rmax = 0, nnz = 0;
    for (uint64_t g = 0; g < nb; g++) rmax = std::max<uint64_t>(rmax, tb_rows[g + 1] - tb_rows[g]);
    for (uint64_t g = 0; g < nb; g++) nnz += row_ptr[tb_rows[g + 1]] - row_ptr[tb_rows[g]];
    if (rmax == 0 || rmax > 64) { why = "BMTBs of 1..64 rows only"; return false; }
    const uint32_t RT = (uint32_t)((rmax + 15) / 16);
    if (nnz == 0 || (double)nb * 16 * RT * K > (double)max_fill * nnz) {
        why = "row blocks too sparse for dense tiles";
        return false;
    }
    // every workgroup streams all of B through LDS: with short row blocks that
    // traffic outgrows A's (R = 4 on C2: 13x) and the gather kernels win
    if ((double)nb * K * N * 2 > 6.0 * 4.0 * nnz && max_fill < (1 << 20)) {
        why = "row blocks too short: B traffic per row block exceeds A's";
        return false;
    }
    for (uint32_t lg = 10; lg >= 8; lg--) {
        const uint64_t KC = 1ull << lg;
        if ((rmax + 1) * (KC + 16) > 65536 || mfma_lds_bytes(lg, CT, (uint32_t)rmax) > lds_budget) continue;
        const uint64_t nc = (K + KC - 1) / KC;
        uint64_t gmax = 0;
        std::vector<uint64_t> cnt(nc);
        for (uint64_t g = 0; g < nb; g++) {
            std::fill(cnt.begin(), cnt.end(), 0);
            for (uint64_t e = row_ptr[tb_rows[g]]; e < row_ptr[tb_rows[g + 1]]; e++) cnt[col[e] >> lg]++;
            for (uint64_t j = 0; j < nc; j++) gmax = std::max(gmax, (cnt[j] + 7) / 8);
        }
        if (gmax > 2ull * kMfmaAThreads || nc > 63) continue;
        if (((KC * 32 * CT) / 16) % kMfmaBThreads) continue;  // whole B units per B thread
        if ((KC * 32 * CT) / 16 / kMfmaBThreads > 8) continue;  // register budget of the B sets
        // the compute waves' partial tiles must fit LDS for the final reduction
        if ((size_t)gsk::kMfmaCompute * RT * CT * 1024 > mfma_lds_bytes(lg, CT, (uint32_t)rmax)) continue;
        t.lgKC = lg; t.nc = (uint32_t)nc; t.RT = RT; t.RMAX = (uint32_t)rmax;
        t.MAXA = gmax <= kMfmaAThreads ? 1 : 2;
        t.gmax = (uint32_t)gmax;
        t.lds_bytes = mfma_lds_bytes(lg, CT, (uint32_t)rmax);
        break;
    }
    if (!t.lgKC) { why = "no chunk width fits LDS and the stage buffers"; return false; }
    const uint32_t KC = 1u << t.lgKC;
    t.seg_start.assign(1, 0);
    std::vector<uint64_t> cur;
    std::vector<uint16_t> pos, hv;
    for (uint64_t g = 0; g < nb; g++) {
        const uint64_t r0 = tb_rows[g], R = tb_rows[g + 1] - r0;
        cur.assign(R, 0);
        for (uint64_t i = 0; i < R; i++) cur[i] = row_ptr[r0 + i];
        for (uint32_t j = 0; j < t.nc; j++) {
            const uint64_t lim = (uint64_t)(j + 1) * KC;
            pos.clear();
            hv.clear();
            for (uint64_t i = 0; i < R; i++) {
                uint64_t e = cur[i];
                for (; e < row_ptr[r0 + i + 1] && col[e] < lim; e++) {
                    // halfword index in the dense image (row stride RS = 2*KC + 32 bytes)
                    pos.push_back((uint16_t)(i * (KC + 16) + (col[e] - (uint64_t)j * KC)));
                    hv.push_back(f32_to_f16_bits(vals[e]));
                }
                cur[i] = e;
            }
            bank_order_segment(pos, hv, (uint32_t)(R * (KC + 16)), t.pos, t.val);
            t.seg_start.push_back((uint32_t)(t.pos.size() / 8));
        }
    }
    t.pos.insert(t.pos.end(), 8, 0);  // spare group: idle lanes' branch-free loads
    t.val.insert(t.val.end(), 8, 0);
    return true;
}

// ------------------------------------------------------------------ k_mfma_ks layout
// Upload layout of k_mfma_ks (kernel_lib.hpp): the K range is split into S ranges of
// KR = 32*NS columns; for every (BMTB g, range q, 32-column k-step s) -- unit u = g*S + q --
// the entries of g's rows in the step's columns, in groups of 8: pos = halfword index in a
// wave image of 96-B rows (local_row*48 + column - step base), val = f16.  The steps'
// groups lie back to back in (u, s) order; steps[2*(u*NS + s)] = the step's first group,
// steps[2*(u*NS + s) + 1] = its group count (at most GCAP, the plan's largest: it sets
// MAXG).  A group's unused entries write 0 into the image's zero row 16*RT.  One spare
// group follows (an empty last step's loads).  The entry order inside a step is
// bank-ordered for the scatter.  (Round 3 padded every step to GCAP groups so that no
// address waited on a load: 1.19-1.35x the algorithmic bytes on the headline layer,
// profiles/traffic_c5h.json.)



bool build_ks_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                    const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                    int64_t s_cfg, int64_t min_rows, int64_t max_fill, ks_tiles &t, std::string &why) {
    const uint64_t nb = tb_rows.size() - 1;
    if (nb == 0 || K == 0) { why = "empty plan"; return false; }
    if (N == 0 || N % 8 != 0) { why = "N must be a multiple of 8"; return false; }
    // KS_WAVES = 16: twice the waves (more loads in flight per CU) when their stages fit LDS
    uint32_t W = kKsWaves;
    uint64_t rmax = 0;
    for (uint64_t g = 0; g < nb; g++) rmax = std::max<uint64_t>(rmax, tb_rows[g + 1] - tb_rows[g]);
    if (rmax < (uint64_t)std::max<int64_t>(1, min_rows) || rmax > 128) { why = "row blocks outside the k_mfma_ks range"; return false; }
    const uint32_t RT = std::max<uint32_t>(2, (uint32_t)((rmax + 15) / 16));  // kernels built for RT 2..8
    const uint32_t CT = ks_ct_rt(N, RT);
    t.CT = CT;
    // (RT 6..8 -- 96..128-row blocks: whole CU rounds on the OPT-30B shapes -- for tiles of
    // at most 32 columns: RT x CT accumulators of 4 VGPRs)
    if (RT > 5 && CT > 2) { why = "row blocks over 80 rows at N > 32"; return false; }
    if (get_config().KS_WAVES == 16 && CT <= 4 && gsk::ks_lds_bytes(CT, RT, 16) <= 160 * 1024) W = 16;
    // KS_WAVES = 4 (N = 32): 256-thread workgroups with the overlapped LDS layout, two per CU, so one
    // workgroup's prologue and combine overlap the other's loop (grouped multi-round launches)
    if (get_config().KS_WAVES == 4 && CT == 2) W = 4;
    // KS_WAVES = 12 (N = 32, RT <= 5, experiments): three waves per SIMD, the stages and the apart
    // partial tiles still within 160 KB (C2 40-row blocks: 155 KB)
    if (get_config().KS_WAVES == 12 && CT == 2 && RT <= 5 && gsk::ks_lds_bytes(CT, RT, 12) <= 160 * 1024) W = 12;
    const uint64_t nnz = row_ptr[tb_rows[nb]] - row_ptr[tb_rows[0]];
    if (nnz == 0 || (double)nb * 16 * RT * K > (double)max_fill * nnz) {  // as build_mfma_tiles
        why = "row blocks too sparse for dense tiles";
        return false;
    }
    // KS_APART: the overlapped layout (0) is built for N = 32 and row tiles 2..5; auto (-1) keeps the
    // apart layout only when it holds as many workgroups per CU as the overlapped one
    {
        const int64_t ap = get_config().KS_APART;
        const bool can_overlap = CT == 2 && ((RT <= 5 && W == kKsWaves) || W == 4);
        const size_t la = gsk::ks_lds_bytes(CT, RT, W, true), lo = gsk::ks_lds_bytes(CT, RT, W, false);
        t.AP = W != 4 && (!can_overlap || ap > 0 || (ap < 0 && (160u * 1024u) / la >= (160u * 1024u) / lo));
    }
    t.lds_bytes = gsk::ks_lds_bytes(CT, RT, W, t.AP);
    if (t.lds_bytes > 160 * 1024) { why = "k_mfma_ks wave stages exceed LDS"; return false; }
    t.RT = RT;
    t.RMAX = (uint32_t)rmax;
    t.W = W;
    // KS_POS8 (8-bit positions in 8 x 16 segments; N = 32, RT <= 8: segment ids < 32)
    t.P8 = get_config().KS_POS8 && CT == 2 && (W == kKsWaves || W == 4);
    t.NT = (CT == 2 || CT == 8) && (W == kKsWaves || W == 12) && !t.P8 && t.AP && get_config().KS_NT ? 1u : 0u;
    // pass 1: the largest step (entries of a row block in 32 columns; P8: groups per segment)
    uint64_t gmax = 1;
    {
        const uint32_t nsg = 4 * RT;
        std::vector<uint32_t> cnt((size_t)((K + 31) / 32) * (t.P8 ? nsg : 1u));
        for (uint64_t g = 0; g < nb; g++) {
            std::fill(cnt.begin(), cnt.end(), 0u);
            for (uint64_t r = tb_rows[g]; r < tb_rows[g + 1]; r++)
                for (uint64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) {
                    const uint64_t st = col[e] / 32;
                    if (t.P8)
                        cnt[st * nsg + ((r - tb_rows[g]) / 8) * 2 + (col[e] % 32) / 16]++;
                    else
                        cnt[st]++;
                }
            if (t.P8) {
                for (size_t st = 0; st < cnt.size() / nsg; st++) {
                    uint64_t ngs = 0;
                    for (uint32_t k = 0; k < nsg; k++) ngs += (cnt[st * nsg + k] + 7) / 8;
                    gmax = std::max<uint64_t>(gmax, ngs);
                }
            } else {
                for (uint32_t c : cnt) gmax = std::max<uint64_t>(gmax, (c + 7) / 8);
            }
        }
    }
    t.GCAP = (uint32_t)gmax;
    t.MAXG = gmax <= 64 ? 1 : (gmax <= 128 ? 2 : (gmax <= 192 ? 3 : (gmax <= 256 ? 4 : 0)));
    if (!t.MAXG) { why = "a k-step holds more than 256 entry groups"; return false; }
    if (t.CT == 8 && !ks_ct8_fits(RT, t.MAXG)) {  // a 128-column instantiation that would spill: 64-column tiles
        t.CT = 4;
        t.NT = 0;  // (KS_NT is built for 32- and 128-column tiles)
        t.lds_bytes = gsk::ks_lds_bytes(4, RT, W, t.AP);
    }
    if (!t.AP && t.MAXG > 2 && W != 4) {  // the 8-wave overlapped layout is instantiated for MAXG <= 2 only
        t.AP = true;
        t.lds_bytes = gsk::ks_lds_bytes(t.CT, RT, W, true);
        if (t.lds_bytes > 160 * 1024) { why = "k_mfma_ks wave stages exceed LDS"; return false; }
    }
    // K ranges (auto): enough workgroups for the 256 CUs over row blocks x column tiles (the grid's
    // y dimension: N = 128 on 64-column tiles is two) -- each workgroup reads only its range's B rows,
    // and a split past one CU round adds B rows per CU and a slab combine without filling more CUs
    // (C2 N = 128, 80-row blocks: 2 K ranges x 2 column tiles 21.5 us, 4 K ranges 33.4 us; r06x)
    {
        const uint64_t ctiles = ks_col_tiles_ct(N, t.CT);
        uint64_t S = s_cfg > 0 ? (uint64_t)s_cfg : std::min<uint64_t>(8, (256 + nb * ctiles - 1) / (nb * ctiles));
        S = std::max<uint64_t>(1, std::min<uint64_t>(S, (K + 31) / 32));
        const uint64_t KR = ((K + S - 1) / S + 31) / 32 * 32;
        t.S = (uint32_t)((K + KR - 1) / KR);
        t.NS = (uint32_t)(KR / 32);
    }
    const uint64_t S = t.S, KR = (uint64_t)t.NS * 32;
    // head steps (ks_tiles::GH): used when padding them to the largest costs at most 6% more groups
    const uint32_t HS = std::min<uint32_t>(W * kKsDepth, t.NS);  // head slots per unit
    if (!t.P8 && get_config().KS_HEAD) {
        uint64_t gh = 1, head_groups = 0, all_groups = 0;
        std::vector<uint32_t> c2((size_t)S * t.NS);
        for (uint64_t g = 0; g < nb; g++) {
            std::fill(c2.begin(), c2.end(), 0u);
            for (uint64_t r = tb_rows[g]; r < tb_rows[g + 1]; r++)
                for (uint64_t e = row_ptr[r]; e < row_ptr[r + 1]; e++) c2[col[e] / 32]++;
            for (size_t st = 0; st < c2.size(); st++) {
                const uint64_t ng = (c2[st] + 7) / 8;
                all_groups += ng;
                if (st % t.NS < HS) {
                    head_groups += ng;
                    gh = std::max(gh, ng);
                }
            }
        }
        const uint64_t padded = (uint64_t)nb * S * HS * gh;
        if ((double)(padded - head_groups) <= 0.06 * (double)all_groups && (double)padded < 2.0e9) t.GH = (uint32_t)gh;
    }
    // 32-bit group and step indices (packed steps: about nnz / 8 + nb*S*NS groups; checked
    // exactly after the build): too large a plan falls back to another kernel
    if ((double)(row_ptr[tb_rows[nb]] - row_ptr[tb_rows[0]]) / 8.0 + (double)nb * S * t.NS * 2.0 >= 4.0e9) {
        why = "k_mfma_ks layout exceeds 32-bit group indices";
        return false;
    }
    const uint32_t RS = gsk::kKsStride / 2;  // halfwords per image row
    const uint32_t pad_h = 16 * RT * RS;      // the zero row
    if (t.P8)
        t.pos8.reserve(row_ptr[tb_rows[nb]] - row_ptr[tb_rows[0]] + (size_t)nb * S * t.NS * 8 * RT + 8);
    else
        t.pos.reserve(row_ptr[tb_rows[nb]] - row_ptr[tb_rows[0]] + (size_t)nb * S * t.NS * 8 + 8);
    t.val.reserve(t.P8 ? t.pos8.capacity() : t.pos.capacity());
    t.steps.reserve((size_t)nb * S * t.NS * 2);
    if (t.GH) {  // the head region first: every slot a zero-row group until its step fills it
        t.pos.assign((size_t)nb * S * HS * t.GH * 8, (uint16_t)pad_h);
        t.val.assign(t.pos.size(), 0);
    }
    std::vector<uint64_t> cur;
    std::vector<uint16_t> pos, hv, prow, pcol, hpos, hval;
    for (uint64_t g = 0; g < nb; g++) {
        const uint64_t r0 = tb_rows[g], R = tb_rows[g + 1] - r0;
        cur.assign(R, 0);
        for (uint64_t i = 0; i < R; i++) cur[i] = row_ptr[r0 + i];
        for (uint64_t q = 0; q < S; q++)
            for (uint32_t s = 0; s < t.NS; s++) {
                const uint64_t base = q * KR + 32ull * s, lim = base + 32;
                pos.clear();
                hv.clear();
                prow.clear();
                pcol.clear();
                for (uint64_t i = 0; i < R; i++) {
                    uint64_t e = cur[i];
                    for (; e < row_ptr[r0 + i + 1] && col[e] < lim; e++) {
                        pos.push_back((uint16_t)(i * RS + (col[e] - base)));
                        prow.push_back((uint16_t)i);
                        pcol.push_back((uint16_t)(col[e] - base));
                        hv.push_back(f32_to_f16_bits(vals[e]));
                    }
                    cur[i] = e;
                }
                size_t before, ng;
                if (t.GH && s < HS) {  // a head step: its fixed slot
                    hpos.clear();
                    hval.clear();
                    bank_order_segment(pos, hv, pad_h, hpos, hval, RS / 2);
                    ng = hpos.size() / 8;
                    GS_CHECK(ng <= t.GH, "k_mfma_ks head step exceeds its slot");
                    before = (((size_t)g * S + q) * HS + s) * t.GH * 8;
                    std::copy(hpos.begin(), hpos.end(), t.pos.begin() + before);
                    std::copy(hval.begin(), hval.end(), t.val.begin() + before);
                } else if (t.P8) {
                    before = t.pos8.size();
                    ng = pos8_step(prow, pcol, hv, RS, t.pos8, t.val);
                } else {
                    before = t.pos.size();
                    bank_order_segment(pos, hv, pad_h, t.pos, t.val, RS / 2);  // pads stay inside the zero row
                    ng = (t.pos.size() - before) / 8;
                }
                GS_CHECK(ng <= t.GCAP, "k_mfma_ks step exceeds its capacity");
                t.steps.push_back((uint32_t)(before / 8));
                t.steps.push_back((uint32_t)ng);
            }
    }
    if (t.P8)
        t.pos8.insert(t.pos8.end(), 8, (uint8_t)0);  // spare group: loads past a wave's last step (never scattered)
    else
        t.pos.insert(t.pos.end(), 8, (uint16_t)pad_h);  // spare group: loads past a wave's last step
    t.val.insert(t.val.end(), 8, 0);
    return true;
}

// ------------------------------------------------------------------ bitmap records
// k_mfma_bm (kernel_lib.hpp): see bm_tiles.  Row blocks of up to 96 rows (RT <= 6 mask
// bytes per record); K split into S ranges of whole k-steps so nb * S workgroups cover
// the CUs (s_cfg > 0: that many).
bool build_bm_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint32_t> &row_ptr,
                    const std::vector<uint64_t> &col, const std::vector<float> &vals, uint64_t K, uint32_t N,
                    int64_t s_cfg, int64_t waves, int64_t max_fill, bm_tiles &t, std::string &why) {
    const uint64_t nb = tb_rows.size() - 1;
    if (nb == 0 || K == 0) { why = "empty plan"; return false; }
    if (N == 0 || N % 8 != 0) { why = "N must be a multiple of 8"; return false; }
    uint64_t rmax = 0;
    for (uint64_t g = 0; g < nb; g++) rmax = std::max<uint64_t>(rmax, tb_rows[g + 1] - tb_rows[g]);
    if (rmax == 0 || rmax > 96) { why = "row blocks outside the k_mfma_bm range (1..96 rows)"; return false; }
    const uint32_t RT = (uint32_t)((rmax + 15) / 16);
    const uint64_t nnz = row_ptr[tb_rows[nb]] - row_ptr[tb_rows[0]];
    if (nnz == 0 || (double)nb * 16 * RT * K > (double)max_fill * nnz) {
        why = "row blocks too sparse for dense tiles";
        return false;
    }
    const bool kb = get_config().BM_KB;
    const uint32_t W = kb || waves != 4 ? 8u : 4u;
    uint64_t S = s_cfg > 0 ? (uint64_t)s_cfg
                           : kb ? std::min<uint64_t>(8, (256 + nb - 1) / nb) : std::max<uint64_t>(1, std::min<uint64_t>(8, 256 / nb));
    S = std::max<uint64_t>(1, std::min<uint64_t>(S, (K + 31) / 32));
    const uint64_t KR = ((K + S - 1) / S + 31) / 32 * 32;
    S = (K + KR - 1) / KR;
    t.S = (uint32_t)S;
    t.NS = (uint32_t)(KR / 32);
    t.RT = RT;
    t.RMAX = (uint32_t)rmax;
    t.W = W;
    t.lds_bytes = gsk::bm_lds_bytes(ks_ct(N), RT, W);
    // k_mfma_bm2 when the range's B slice fits LDS next to the selector table
    const size_t slice = 128u + (size_t)t.NS * 32u * 32u * ks_ct(N);
    t.kb = kb;
    t.v2 = !kb && get_config().BM_V2 && slice <= 160u * 1024u;
    if (t.v2) {
        t.lds_bytes = slice;
        t.W = RT;
    }
    const uint64_t nrec = nb * S * t.NS * 64;
    GS_CHECK(nrec < (1ull << 31), "k_mfma_bm layout exceeds 31-bit record indices");
    t.rec.assign(nrec * 2, 0u);
    auto rec_of = [&](uint64_t g, uint64_t i, uint64_t c, uint32_t &tt, uint32_t &bit) -> uint64_t {
        const uint64_t qq = c / KR, cc = c % KR, st = cc / 32, w = cc % 32;
        tt = (uint32_t)(i / 16);
        bit = (uint32_t)(w % 8);
        const uint64_t lane = (w / 8) * 16 + i % 16;
        return ((g * S + qq) * t.NS + st) * 64 + lane;
    };
    auto mask_byte = [&](uint64_t r, uint32_t tt) -> uint32_t {
        return tt < 4 ? (t.rec[2 * r] >> (8 * tt)) & 0xffu : (t.rec[2 * r + 1] >> (8 * (tt - 4))) & 0xffu;
    };
    for (uint64_t g = 0; g < nb; g++)
        for (uint64_t i = 0; i < tb_rows[g + 1] - tb_rows[g]; i++)
            for (uint64_t e = row_ptr[tb_rows[g] + i]; e < row_ptr[tb_rows[g] + i + 1]; e++) {
                uint32_t tt, bit;
                const uint64_t r = rec_of(g, i, col[e], tt, bit);
                if (tt < 4) t.rec[2 * r] |= 1u << (8 * tt + bit);
                else t.rec[2 * r + 1] |= 1u << (8 * (tt - 4) + bit);
            }
    // step bases and lane offsets (lane after lane, tile after tile)
    const uint64_t nst = nb * S * t.NS;
    t.sbase.assign(nst + 1, 0u);
    uint64_t run = 0;
    std::vector<uint32_t> lane_pre(nrec, 0);  // values before (lane, tile 0) within the step
    for (uint64_t x = 0; x < nst; x++) {
        GS_CHECK(run < (1ull << 32) - 64, "k_mfma_bm values exceed 32-bit offsets");
        t.sbase[x] = (uint32_t)run;
        uint32_t off = 0;
        for (uint32_t l = 0; l < 64; l++) {
            const uint64_t r = x * 64 + l;
            lane_pre[r] = off;
            t.rec[2 * r + 1] |= off << 16;
            for (uint32_t tt = 0; tt < RT; tt++) off += (uint32_t)__builtin_popcount(mask_byte(r, tt));
        }
        GS_CHECK(off < 65536u, "k_mfma_bm step holds more than 65535 values");
        run += off;
    }
    t.sbase[nst] = (uint32_t)run;
    t.val.assign(run + 16, 0);
    if (kb) {
        // k_mfma_kb fetches a step's run in whole 16-B units from its aligned start: NVB KB
        uint64_t umax = 1;
        for (uint64_t x = 0; x < nst; x++) umax = std::max<uint64_t>(umax, (t.sbase[x + 1] - (t.sbase[x] & ~7u) + 7) / 8);
        t.NVB = (uint32_t)((umax + 63) / 64);
        if (t.NVB == 3) t.NVB = 4;
        if (t.NVB > 4) { why = "a k-step holds more than 4 KB of values (k_mfma_kb)"; return false; }
        t.lds_bytes = gsk::kb_lds_bytes(ks_ct(N), RT, W, t.NVB);
        if (t.lds_bytes > 160 * 1024) { why = "k_mfma_kb slots exceed LDS"; return false; }
    }
    for (uint64_t g = 0; g < nb; g++)
        for (uint64_t i = 0; i < tb_rows[g + 1] - tb_rows[g]; i++)
            for (uint64_t e = row_ptr[tb_rows[g] + i]; e < row_ptr[tb_rows[g] + i + 1]; e++) {
                uint32_t tt, bit;
                const uint64_t r = rec_of(g, i, col[e], tt, bit);
                uint64_t pos = t.sbase[r / 64] + lane_pre[r];
                for (uint32_t t2 = 0; t2 < tt; t2++) pos += (uint32_t)__builtin_popcount(mask_byte(r, t2));
                pos += (uint32_t)__builtin_popcount(mask_byte(r, tt) & ((1u << bit) - 1u));
                t.val[pos] = f32_to_f16_bits(vals[e]);
            }
    return true;
}

// ------------------------------------------------------------------ 2:4 panels
// Block layout of k_nm_mfma (kernel_lib.hpp) from the plan's COO: every row is
// cut into 64-column k-steps (the col-direction BMTs of a 2:4 row: 32 entries
// each), every aligned group of four columns keeps its (at most two) entries as
// two values + two 2-bit positions.  Duplicate coordinates (col padding of the
// plan, value 0) are summed.  Returns false (and why) when a group holds more
// than two distinct columns or the panels would store over twice the entries
// (beyond 4M value slots).
// T = 16-row tiles per k_nm_mfma workgroup (nm_tiles): its two wave sets hold G0 = ceil(T/2)
// and G1 = T/2 tiles; per (workgroup w, set rh, k-step s) one block of 512 B of positions +
// G_rh KB of values at w * S * nm_wg_block_bytes(T) + rh * S * (512 + 1024 G0) + s * (512 + 1024
// G_rh).  T = 8 is the 64-row-group layout (group g = 2w + rh at g * S * 4608), rounded to whole
// 256-row blocks as k_nm_mfma_ks / k_nm_mfma4 read it.
bool build_nm_panels(const std::vector<uint64_t> &rows, const std::vector<uint64_t> &col, const universal_array &vals,
                     uint64_t row_num, uint64_t K, std::vector<unsigned char> &blk, uint32_t &S, std::string &why,
                     uint32_t T) {
    const uint64_t nnz = col.size();
    if (row_num == 0 || K == 0 || nnz == 0) { why = "empty sub-matrix"; return false; }
    if (T < 2 || T > 8) { why = "2..8 tiles per workgroup"; return false; }
    const uint64_t S64 = (K + gsk::kNmKC - 1) / gsk::kNmKC * 4;  // k-steps, whole 256-column chunks
    const uint64_t rows_wg = 16ull * T;
    const uint64_t nwg = T == 8 ? (row_num + 255) / 256 * 2 : (row_num + rows_wg - 1) / rows_wg;
    const uint64_t G0 = (T + 1) / 2, WB = gsk::nm_wg_block_bytes(T);
    const double slots = (double)nwg * (double)rows_wg * (double)S64 * 32.0;
    if (slots > 2.0 * (double)nnz && slots > (double)(1 << 22)) {  // small plans always qualify
        why = "2:4 panels would store over twice the entries";
        return false;
    }
    if (S64 > 0xffffffffull || nwg * S64 * WB > (1ull << 40)) { why = "too large"; return false; }
    std::vector<uint64_t> rp(row_num + 1, 0);
    for (uint64_t r : rows) {
        if (r >= row_num) { why = "row index beyond row count"; return false; }
        rp[r + 1]++;
    }
    for (uint64_t i = 0; i < row_num; i++) rp[i + 1] += rp[i];
    std::vector<uint64_t> cur(rp.begin(), rp.end() - 1), ord(nnz);
    for (uint64_t e = 0; e < nnz; e++) ord[cur[rows[e]]++] = e;
    // block of (workgroup w, set rh, k-step s)
    auto block = [&](uint64_t w, uint64_t rh, uint64_t s) {
        return blk.data() + w * S64 * WB + rh * S64 * (512 + 1024 * G0) + s * (512 + 1024 * (rh ? T / 2 : G0));
    };
    blk.assign(nwg * S64 * WB, 0);
    for (uint64_t w = 0; w < nwg; w++)  // default positions (0, 1) in every group
        for (uint64_t rh = 0; rh < 2; rh++)
            for (uint64_t s = 0; s < S64; s++) {
                uint16_t *ix = reinterpret_cast<uint16_t *>(block(w, rh, s));
                for (int i = 0; i < 256; i++) ix[i] = 0x4444;
            }
    const uint64_t Kp = S64 * 64;
    std::vector<float> dv(Kp, 0.f);
    std::vector<uint8_t> has(Kp, 0);
    for (uint64_t r = 0; r < row_num; r++) {
        if (rp[r] == rp[r + 1]) continue;
        for (uint64_t e = rp[r]; e < rp[r + 1]; e++) {
            const uint64_t c = col[ord[e]];
            if (c >= K) { why = "column index beyond column count"; return false; }
            has[c] = 1;
            dv[c] += (float)vals.read_float_from_arr(ord[e]);
        }
        const uint64_t w = r / rows_wg, within = r % rows_wg, rh = within >= 16 * G0 ? 1 : 0;
        const uint64_t rt = (within - rh * 16 * G0) / 16, rr = r % 16;
        for (uint64_t gi = 0; gi < Kp / 4; gi++) {
            int pos[2], n = 0;
            for (int p = 0; p < 4; p++)
                if (has[4 * gi + p]) {
                    if (n == 2) {
                        why = "a row holds more than two entries in an aligned group of four columns (not 2:4)";
                        return false;
                    }
                    pos[n++] = p;
                }
            if (n == 0) continue;
            if (n == 1) pos[1] = pos[0] == 3 ? 2 : 3;  // zero partner at another position
            const int lo = std::min(pos[0], pos[1]), hi = std::max(pos[0], pos[1]);
            const uint64_t s = gi / 16, j = gi % 16, g = j / 4, sg = j % 4, lane = g * 16 + rr;
            unsigned char *b = block(w, rh, s);
            uint16_t *v = reinterpret_cast<uint16_t *>(b + 512 + rt * 1024 + lane * 16) + sg * 2;
            v[0] = has[4 * gi + lo] ? f32_to_f16_bits(dv[4 * gi + lo]) : 0;
            v[1] = has[4 * gi + hi] ? f32_to_f16_bits(dv[4 * gi + hi]) : 0;
            uint16_t *ix = reinterpret_cast<uint16_t *>(b + lane * 8) + rt;
            *ix = (uint16_t)((*ix & ~(0xfu << (4 * sg))) | ((unsigned)(lo | (hi << 2)) << (4 * sg)));
        }
        for (uint64_t e = rp[r]; e < rp[r + 1]; e++) {
            has[col[ord[e]]] = 0;
            dv[col[ord[e]]] = 0.f;
        }
    }
    S = (uint32_t)S64;
    return true;
}

uint32_t nm_tiles_for(uint64_t row_num, int64_t cfg_tiles, uint32_t N) {
    if (cfg_tiles > 0) {
        GS_CHECK(cfg_tiles == 2 || cfg_tiles == 4 || cfg_tiles == 7 || cfg_tiles == 8, "NM_TILES: 2, 4, 7 or 8");
        return (uint32_t)cfg_tiles;
    }
    const uint64_t tiles = (row_num + 15) / 16;
    uint32_t best = 8;
    uint64_t best_load = ~0ull;
    for (uint32_t T : {8u, 7u, 4u, 2u}) {
        // N = 128: B (1.8 MB per workgroup at K = 7168) is two thirds of a CU's intake, and 256
        // workgroups of 7 tiles ran 2% slower than 224 of 8 (profiles/r06c_ab_c3.txt); at N <= 64
        // the 7-tile grid is 2-4% faster
        if (T == 7 && N >= 128) continue;
        const uint64_t wgs = T == 8 ? (row_num + 255) / 256 * 2 : (tiles + T - 1) / T;
        const uint64_t load = (wgs + 255) / 256 * T;  // tiles per CU, one workgroup per CU at a time
        if (load < best_load) {
            best_load = load;
            best = T;
        }
    }
    return best;
}

mc_layout choose_matrix_core_layout(const meta_data_set &m, const kernel_spec &sp, int sb, uint64_t K, int dtype) {
    mc_layout L;
    const config_t cfg = get_config();
    const int64_t Nd = cfg.DENSE_MATRIX_SIZE;
    L.N = (uint32_t)std::max<int64_t>(0, Nd);
    if (dtype != 1) { L.why = "fp32 plan"; return L; }
    const uint64_t row_num = row_num_of_sub_matrix(m, sb);
    const auto &rows = m.u(GLOBAL_META, "nz_row_indices", sb);
    if (sp.family == KF_ROW_CHUNKS && !sp.interleaved && cfg.NM_MFMA && (Nd == 8 || Nd == 16 || Nd == 32 || Nd == 64 || Nd == 128)) {
        // col-direction BMTs that are 2:4 panels: sparse matrix cores, self-contained blocks
        const auto &col = m.u(GLOBAL_META, "nz_col_indices", sb);
        auto vals = m.get_element(GLOBAL_META, "nz_vals", sb)->meta_data_arr;
        // the experiments-build 256-row kernels read the T = 8 layout only
        const bool v256 = cfg.NM_KS != 0 || cfg.NM_V4 != 0;
        L.nm_T = v256 ? 8u : nm_tiles_for(row_num, cfg.NM_TILES, L.N);
        if (build_nm_panels(rows, col, *vals, row_num, K, L.nm_blk, L.nm_S, L.why, L.nm_T)) {
            L.kind = mc_layout::NM;
            L.nm_rows = row_num;
            // k_nm_mfma_ks (NM_KS): 256-row workgroups, K split so they cover the CUs
            const uint32_t nch = L.nm_S / 4, nb = (uint32_t)((row_num + 255) / 256);
            uint32_t sp = cfg.NM_SPLIT > 0 ? (uint32_t)cfg.NM_SPLIT : std::max<uint32_t>(1, 256 / std::max<uint32_t>(nb, 1));
            sp = std::max(1u, std::min(sp, nch));
            L.nm_ks = cfg.NM_KS != 0 && Nd >= 16;
            L.nm4 = !L.nm_ks && K % gsk::kNmKC == 0 && nch >= 2 &&
                    ((cfg.NM_V4 > 0 && (Nd == 64 || Nd == 128)) || (cfg.NM_V4 < 0 && Nd == 128));
            L.nm_nt = cfg.NM_NT != 0 && !L.nm_ks && !L.nm4;
            L.nm_ncs = (nch + sp - 1) / sp;
            L.nm_split = (nch + L.nm_ncs - 1) / L.nm_ncs;
        }
        return L;
    }
    if (!cfg.MFMA_TILES || !m.is_exist(TBLOCK_META, "first_row_indices", sb) ||
        !(sp.family == KF_BLOCK_TOTAL || (sp.family == KF_WARP_TOTAL && sp.tblock_parent))) {
        L.why = "no fp16 BMTB row blocks";
        return L;
    }
    const auto &col = m.u(GLOBAL_META, sp.interleaved ? "nz_col_indices_after_interlance_storage" : "nz_col_indices", sb);
    auto vals = m.get_element(GLOBAL_META, sp.interleaved ? "nz_vals_after_interlance_storage" : "nz_vals", sb)->meta_data_arr;
    std::vector<uint32_t> rp0(row_num + 1, 0);
    for (uint64_t r : rows) {
        GS_CHECK(r < row_num, "row index beyond row count");
        rp0[r + 1]++;
    }
    for (uint64_t i = 0; i < row_num; i++) rp0[i + 1] += rp0[i];
    L.tbr = m.u(TBLOCK_META, "first_row_indices", sb);
    const canon_rows cr = canonical_rows(rp0, col, *vals);
    const uint32_t N = (uint32_t)Nd;
    if (cfg.MFMA_BM && build_bm_tiles(L.tbr, cr.rp, cr.col, cr.val, K, N, cfg.BM_SPLIT, cfg.BM_WAVES,
                                      cfg.MFMA_MAX_FILL, L.bm, L.why)) {
        L.kind = mc_layout::BM;
        return L;
    }
    if (cfg.MFMA_KS &&
        build_ks_tiles(L.tbr, cr.rp, cr.col, cr.val, K, N, cfg.KS_SPLIT, cfg.KS_MIN_ROWS, cfg.MFMA_MAX_FILL, L.ks, L.why)) {
        L.kind = mc_layout::KS;
        return L;
    }
    // k_mfma_rows: its variant from the config, fixed here
    const int64_t gl = cfg.MFMA_GLDS;
    L.rows_glds = gl >= 4 ? 4 : (gl ? 2 : 0);
    L.rows_wct = (gl == 1 && cfg.MFMA_COMPUTE_WAVES == 8) ? 8 : gsk::kMfmaCompute;
    const size_t budget = (size_t)std::min<int64_t>(cfg.SHARED_MEM_TOTAL_SIZE, 160 * 1024);
    if (!build_mfma_tiles(L.tbr, cr.rp, cr.col, cr.val, K, N, budget, cfg.MFMA_MAX_FILL, L.rows, L.why)) return L;
    L.rows_nbg = 3;
    if (L.rows.lgKC == 8 && gl && gl < 4 && L.rows_wct == gsk::kMfmaCompute)  // deeper B rings fit with 256-column chunks
        L.rows_nbg = cfg.MFMA_GLDS_NBUF >= 5 ? 5 : (cfg.MFMA_GLDS_NBUF == 4 ? 4 : 3);
    const uint32_t nat = 64u * (gsk::kMfmaWaves - L.rows_wct - (L.rows_glds ? (uint32_t)L.rows_glds : (uint32_t)gsk::kMfmaBWaves));
    L.rows_maxa = L.rows.gmax > nat ? 2 : 1;
    L.rows_flags = cfg.MFMA_FLAGS && L.rows_glds == 2 && L.rows_nbg == 3 && L.rows_wct == gsk::kMfmaCompute;
    // K-split: enough workgroups per row block to cover the CUs, at least one chunk each; auto:
    // split only when the row blocks cover under half the CUs (the slab combine costs
    // ~micro-seconds at the tail)
    const uint64_t nb = L.tbr.size() - 1;
    uint32_t ks = cfg.MFMA_KSPLIT > 0 ? (uint32_t)cfg.MFMA_KSPLIT
                                      : (nb >= 128 ? 1u : (uint32_t)std::min<uint64_t>(4, 256 / std::max<uint64_t>(nb, 1)));
    ks = std::max(1u, std::min(ks, L.rows.nc));
    L.rows_ncs = (L.rows.nc + ks - 1) / ks;
    L.rows_ksplit = (L.rows.nc + L.rows_ncs - 1) / L.rows_ncs;  // no empty split
    L.kind = mc_layout::ROWS;
    return L;
}

}  // namespace gs
