// device_plan.hip -- uploads a compiled plan to HBM in the layout of its
// kernel family and dispatches the gfx950 kernels of hip_code/kernel_lib.hpp.
#include "../hip_code/kernel_lib.hpp"
#include "../host/gs_plan.hpp"
#include "../host/index_compress.hpp"
#include "../host/device_layout.hpp"

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>

namespace gs {

#define HIP_OK(x)                                                                                   \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) throw gs_error(std::string(#x) + ": " + hipGetErrorString(e_), -3); \
    } while (0)

namespace {

constexpr uint64_t kPad = 64;  // extra zeroed entries after every A stream

template <class T>
T *dev_copy(device_plan &d, const std::vector<T> &h, uint64_t pad = 0) {
    size_t n = h.size() + pad;
    T *p = nullptr;
    HIP_OK(hipMalloc(&p, std::max<size_t>(n, 1) * sizeof(T)));
    d.allocations.push_back(p);
    if (!h.empty()) HIP_OK(hipMemcpy(p, h.data(), h.size() * sizeof(T), hipMemcpyHostToDevice));
    if (pad) HIP_OK(hipMemset(p + h.size(), 0, pad * sizeof(T)));
    d.bytes_A += h.size() * sizeof(T);
    return p;
}

std::vector<uint32_t> to_u32(const std::vector<uint64_t> &v, const char *what) {
    std::vector<uint32_t> o(v.size());
    for (size_t i = 0; i < v.size(); i++) {
        GS_CHECK(v[i] <= 0xffffffffull, std::string(what) + " exceeds 32 bits");
        o[i] = (uint32_t)v[i];
    }
    return o;
}

// An index array a gather kernel reads through gsk::idx_at.  With MODEL_DRIVEN_COMPRESS and
// an exact formula for it (index_compress.cc; the reference prints the same formulas into its
// kernels, code_generator.cc:2618-3063) nothing is uploaded (linear / branch / cycle kinds) or
// only the narrow residuals are; otherwise the u32 array.  type_ori: the array's compressed
// data type, which bounds the residual width as in the reference's if_residual.
uint32_t *upload_index(device_plan &d, const std::vector<uint64_t> &v, data_type type_ori, const char *what,
                       gsk::idx_formula &f) {
    f = gsk::idx_formula();
    if (get_config().MODEL_DRIVEN_COMPRESS) {
        const index_compression c = analyze_index_compression(v, type_ori, get_config().BRANCH_COMPRESS_MAX_SIZE);
        if (device_formula_of(c, f)) {
            d.index_formulas++;
            if (f.kind == gsk::IDX_RESIDUAL_U8) {
                d.index_bytes_saved += v.size() * 3;
                return (uint32_t *)dev_copy(d, std::vector<uint8_t>(c.res.begin(), c.res.end()), 4);
            }
            if (f.kind == gsk::IDX_RESIDUAL_U16) {
                d.index_bytes_saved += v.size() * 2;
                return (uint32_t *)dev_copy(d, std::vector<uint16_t>(c.res.begin(), c.res.end()), 2);
            }
            d.index_bytes_saved += v.size() * 4;
            return nullptr;
        }
    }
    return dev_copy(d, to_u32(v, what));
}

uint32_t *upload_index(device_plan &d, const meta_data_set &m, POS_TYPE pos, const char *name, int sb,
                       gsk::idx_formula &f) {
    return upload_index(d, m.u(pos, name, sb), m.get_element(pos, name, sb)->meta_data_arr->get_compress_data_type(), name,
                        f);
}

// CSR row pointer of the (possibly padded, row-sorted) COO
std::vector<uint32_t> csr_row_ptr(const std::vector<uint64_t> &row, uint64_t row_num) {
    std::vector<uint32_t> rp(row_num + 1, 0);
    for (uint64_t r : row) {
        GS_CHECK(r < row_num, "row index beyond row count");
        rp[r + 1]++;
    }
    for (uint64_t i = 0; i < row_num; i++) rp[i + 1] += rp[i];
    return rp;
}

uint32_t pow2ceil_u(uint32_t x) {
    uint32_t p = 1;
    while (p < x) p <<= 1;
    return p;
}

// ------------------------------------------------------------------ LDS tiles
// Chunk-major A layout for k_lds_rows (kernel_lib.hpp): for BMTB g and column
// chunk j = [j*KC, (j+1)*KC), the entries of g's rows whose columns fall in the
// chunk, row after row, each row padded to 4 entries (column 0, value 0) and
// the segment padded to 8 entries so it stages as whole 16-B units.
struct lds_tiles {
    uint32_t KC = 0, nc = 0, RSB = 0, rpw_max = 0, seg_cap = 0, waves = 0, maxr = 0;
    size_t lds_bytes = 0;
    std::vector<uint32_t> seg_start, seg_row_off;
    std::vector<uint16_t> tcol;
    std::vector<uint32_t> src;  // source entry per tile entry (~0u: padding)
};

constexpr int kLdsMaxU = 12;  // 16-B staging registers per thread (k_lds_rows MAXU)

// returns false (and the reason) when the plan/shape does not fit the kernel
bool build_lds_tiles(const std::vector<uint64_t> &tb_rows, const std::vector<uint64_t> &tb_bmw,
                     const std::vector<uint64_t> &bmw_rows, const std::vector<uint32_t> &row_ptr,
                     const std::vector<uint64_t> &col, uint64_t K, uint32_t N, uint32_t vbytes, size_t lds_budget,
                     lds_tiles &t, std::string &why, bool dma = false, uint64_t want = 1) {
    const uint64_t nb = tb_rows.size() - 1;
    if (nb == 0 || K == 0) { why = "empty plan"; return false; }
    if ((N * vbytes) % 16 != 0) { why = "B rows are not whole 16-B units"; return false; }
    const uint32_t UB = N * vbytes / 16;
    if (UB > 64 || (UB & (UB - 1))) { why = "16-B units per B row must be a power of two <= 64"; return false; }
    uint32_t waves = 0, maxr = 0, rpw = 0;
    for (uint64_t g = 0; g < nb; g++) {
        const uint64_t w0 = tb_bmw[g], w1 = tb_bmw[g + 1];
        if (w1 <= w0 || bmw_rows[w0] != tb_rows[g] || bmw_rows[w1] != tb_rows[g + 1]) {
            why = "BMWs do not tile their BMTB";
            return false;
        }
        waves = std::max<uint32_t>(waves, (uint32_t)(w1 - w0));
        rpw = std::max<uint32_t>(rpw, (uint32_t)(tb_rows[g + 1] - tb_rows[g]));
        for (uint64_t w = w0; w < w1; w++) maxr = std::max<uint32_t>(maxr, (uint32_t)(bmw_rows[w + 1] - bmw_rows[w]));
    }
    if (waves > 16) { why = "more than 16 BMWs per BMTB"; return false; }
    // BMWs of 5..8 rows: one row per slot (k_lds_rows_rs; fp32 N = 32 by LDS-DMA only)
    const bool rowslot = dma && vbytes == 4 && N == 32 && maxr > 4 && maxr <= 8;
    if (maxr > 4 && !rowslot) { why = "more than 4 rows per BMW"; return false; }
    maxr = maxr <= 1 ? 1 : (maxr <= 2 ? 2 : (maxr <= 4 ? 4 : 8));
    // B rows in LDS at an odd count of 16-B units (bank spread for random rows), except fp32 at
    // N = 32 (8 lanes x 16 B per row, 8 slots per wave): rows at 128 B, so a row starts on bank 0
    // or 32 by its parity, and each row's entries are ordered so that the slots whose B reads
    // share an LDS cycle (ds_read_b128 lane groups: slots {0,3} and {1,2} of each half-wave) read
    // rows of opposite parity -- conflict-free (pair_banks below; r06 PMC: 42% of the LDS cycles
    // were bank conflicts with the odd stride)
    const bool pair_banks = vbytes == 4 && N == 32;
    const uint32_t RSB = pair_banks ? N * vbytes : N * vbytes + (UB % 2 == 0 ? 16u : 0u);
    const uint32_t ebytes = 2 + vbytes;
    const uint64_t nthr = 64ull * waves;
    const uint64_t max_kc = std::min<uint64_t>(K, 65536);
    // smallest chunk count whose largest segment still fits LDS and the staging registers
    uint64_t nc = std::max<uint64_t>(1, (K * RSB * (dma ? 2 : 1) + lds_budget / 2) / (lds_budget * 3 / 4));
    // want > 1 (the plan's K split): past the first chunk count that fits, a few more are tried and
    // the one with the fewest columns in the longest K range is kept -- a range is whole chunks, so
    // 32 chunks in 6 ranges (6+6+6+6+6+2) run 6 chunks of 160 columns where 36 would run 6 of 144
    // (C2 fp32 (64,8): 27.6 -> 25.8 us, profiles/r06zj)
    bool found = false;
    uint64_t nc_first = 0, best_cost = 0;
    for (;; nc++) {
        uint64_t KC = (K + nc - 1) / nc;
        KC = (KC + 7) / 8 * 8;
        if (KC > max_kc) continue;
        if (KC < 64 && nc > 1) {
            if (found) break;
            why = "column chunks would be under 64 rows of B";
            return false;
        }
        const uint64_t ncc = (K + KC - 1) / KC;
        uint64_t cap = 0;
        std::vector<uint64_t> segl(ncc);
        for (uint64_t g = 0; g < nb; g++) {
            std::fill(segl.begin(), segl.end(), 0);
            for (uint64_t r = tb_rows[g]; r < tb_rows[g + 1]; r++) {
                uint64_t e = row_ptr[r];
                while (e < row_ptr[r + 1]) {
                    const uint64_t j = col[e] / KC;
                    uint64_t e1 = e;
                    while (e1 < row_ptr[r + 1] && col[e1] / KC == j) e1++;
                    segl[j] += (e1 - e + 3) / 4 * 4;
                    e = e1;
                }
            }
            for (uint64_t j = 0; j < ncc; j++) cap = std::max(cap, (segl[j] + 7) / 8 * 8);
        }
        const uint64_t lds = KC * RSB + cap * ebytes + (rpw + 1) * 4;
        const uint64_t units = KC * UB + cap * ebytes / 16;
        // k_lds_rows_dma / _rs: two buffers of B rows + columns + values (row offsets by loads)
        const uint64_t buf = KC * RSB + std::max<uint64_t>(cap, 8) * ebytes;
        const bool fits = dma ? 2 * buf <= lds_budget : lds <= lds_budget && units <= (uint64_t)kLdsMaxU * nthr;
        if (fits) {
            const uint64_t w = std::max<uint64_t>(1, std::min<uint64_t>(want, ncc));
            const uint64_t cost = (ncc + w - 1) / w * KC;  // columns of the longest K range
            if (!found || cost < best_cost) {
                t.KC = (uint32_t)KC;
                t.nc = (uint32_t)ncc;
                t.seg_cap = (uint32_t)std::max<uint64_t>(cap, 8);
                t.lds_bytes = dma ? (size_t)(2 * buf + 15) / 16 * 16
                                  : (size_t)(KC * RSB + (uint64_t)t.seg_cap * ebytes + (rpw + 1) * 4 + 15) / 16 * 16;
                best_cost = cost;
            }
            if (!found) {
                found = true;
                nc_first = nc;
            }
        }
        if (found && (want <= 1 || nc >= nc_first + 2 * want)) break;
        if (nc > K) {
            if (found) break;
            why = "no chunking fits LDS";
            return false;
        }
    }
    if (rowslot && (uint64_t)t.KC * RSB > 65536) { why = "row-per-slot chunks over 511 B rows"; return false; }
    t.RSB = RSB;
    t.rpw_max = rpw;
    t.waves = waves;
    t.maxr = maxr;
    t.seg_start.assign(1, 0);
    t.seg_row_off.assign(nb * t.nc * (rpw + 1), 0);
    std::vector<uint64_t> cur(rpw);
    std::vector<uint32_t> slot_of(rpw);  // rowslot: a row's slot = its place in its BMW
    for (uint64_t g = 0; g < nb; g++) {
        const uint64_t r0 = tb_rows[g], nr = tb_rows[g + 1] - r0;
        for (uint64_t i = 0; i < nr; i++) cur[i] = row_ptr[r0 + i];
        if (rowslot)
            for (uint64_t w = tb_bmw[g]; w < tb_bmw[g + 1]; w++)
                for (uint64_t r = bmw_rows[w]; r < bmw_rows[w + 1]; r++) slot_of[r - r0] = (uint32_t)(r - bmw_rows[w]);
        for (uint32_t j = 0; j < t.nc; j++) {
            const uint64_t lim = (uint64_t)(j + 1) * t.KC, base = t.tcol.size();
            uint32_t *off = &t.seg_row_off[(g * t.nc + j) * (rpw + 1)];
            for (uint64_t i = 0; i < nr; i++) {
                off[i] = (uint32_t)(t.tcol.size() - base);
                uint64_t e = cur[i];
                const uint64_t e_end = row_ptr[r0 + i + 1];
                for (; e < e_end && col[e] < lim; e++) {
                    t.tcol.push_back((uint16_t)(col[e] - (uint64_t)j * t.KC));
                    t.src.push_back((uint32_t)e);
                }
                cur[i] = e;
                while ((t.tcol.size() - base) % 4) { t.tcol.push_back(0); t.src.push_back(~0u); }
                if (rowslot) {
                    // slot s reads entry 4i + q of its row in the q-th read of iteration i: slots
                    // {0,1,4,5} take column parity k & 1 at entry k, slots {2,3,6,7} the opposite
                    // (the b128 lane groups pair slots {0,3} and {1,2} of each half-wave)
                    const size_t rs = base + off[i], re = t.tcol.size();
                    const uint32_t ph = (slot_of[i] & 2u) ? 1u : 0u;
                    std::vector<std::pair<uint16_t, uint32_t>> ev, od;
                    for (size_t k = rs; k < re; k++) (t.tcol[k] & 1u ? od : ev).push_back({t.tcol[k], t.src[k]});
                    std::reverse(ev.begin(), ev.end());
                    std::reverse(od.begin(), od.end());
                    for (size_t k = rs; k < re; k++) {
                        const bool want_odd = ((k - rs + ph) & 1u) != 0u;
                        auto &v = (want_odd && !od.empty()) || ev.empty() ? od : ev;
                        t.tcol[k] = v.back().first;
                        t.src[k] = v.back().second;
                        v.pop_back();
                    }
                } else if (pair_banks) {
                    // per 32-entry block of the row (slot s takes entries 4s..4s+3, entry q in the
                    // q-th read): the reads of slots (0,3), (1,2), (4,7), (5,6) at one q get one
                    // even and one odd column while both kinds last (any entry order sums the row)
                    static const int pairs[4][2] = {{0, 3}, {1, 2}, {4, 7}, {5, 6}};
                    const size_t rs = base + off[i], re = t.tcol.size();
                    for (size_t b0 = rs; b0 < re; b0 += 32) {
                        const size_t n = std::min<size_t>(32, re - b0);
                        std::vector<std::pair<uint16_t, uint32_t>> ev, od;
                        for (size_t k = 0; k < n; k++) (t.tcol[b0 + k] & 1u ? od : ev).push_back({t.tcol[b0 + k], t.src[b0 + k]});
                        auto take = [&](bool want_odd) {
                            auto &v = (want_odd && !od.empty()) || ev.empty() ? od : ev;
                            const auto x = v.back();
                            v.pop_back();
                            return x;
                        };
                        for (int q = 0; q < 4; q++)
                            for (const auto &pr : pairs) {
                                const size_t pa = (size_t)pr[0] * 4 + q, pb = (size_t)pr[1] * 4 + q;
                                if (pa < n) {
                                    const auto x = take(ev.size() < od.size());
                                    t.tcol[b0 + pa] = x.first;
                                    t.src[b0 + pa] = x.second;
                                    if (pb < n) {
                                        const auto y = take(!(x.first & 1u));
                                        t.tcol[b0 + pb] = y.first;
                                        t.src[b0 + pb] = y.second;
                                    }
                                } else if (pb < n) {
                                    const auto y = take(false);
                                    t.tcol[b0 + pb] = y.first;
                                    t.src[b0 + pb] = y.second;
                                }
                            }
                    }
                }
            }
            for (uint64_t i = nr; i <= rpw; i++) off[i] = (uint32_t)(t.tcol.size() - base);
            // rowslot: the chunk's columns as LDS byte offsets of their B rows (column x 128 B, < 64 KB
            // for KC <= 511), so the kernel adds its lane's 16-B piece and reads (no shift, no mask)
            if (rowslot)
                for (size_t k = base; k < t.tcol.size(); k++) t.tcol[k] = (uint16_t)(t.tcol[k] * RSB);
            while ((t.tcol.size() - base) % 8) { t.tcol.push_back(0); t.src.push_back(~0u); }
            GS_CHECK(t.tcol.size() - base <= t.seg_cap, "LDS tile segment exceeds its capacity");
            GS_CHECK(t.tcol.size() < 0xffffffffull, "LDS tile layout exceeds 32-bit offsets");
            t.seg_start.push_back((uint32_t)t.tcol.size());
        }
    }
    return true;
}

}  // namespace

// merge-path levels of a compact CSR walked at `work_size` steps of the path (rows consumed +
// nonzeros consumed): level w at diagonal p = w * work_size has consumed j rows (row i is consumed
// at path position ends[i] + i + 1) and p - j nonzeros -- the split the reference's merge-path
// operators produce (get_begin_rows_of_level_after_merge_path.cc), for CSRs the plan never held
// (the column partitions of MP_COL_PARTS)
static void merge_path_levels(const std::vector<uint64_t> &rows, uint64_t row_num, uint64_t work_size,
                              std::vector<uint64_t> &lr, std::vector<uint64_t> &ln) {
    std::vector<uint64_t> cnt(row_num, 0);
    for (uint64_t r : rows) cnt[r]++;
    std::vector<uint64_t> ends, crow;
    uint64_t acc = 0;
    for (uint64_t r = 0; r < row_num; r++)
        if (cnt[r]) {
            acc += cnt[r];
            ends.push_back(acc);
            crow.push_back(r);
        }
    lr.clear();
    ln.clear();
    uint64_t j = 0;
    for (uint64_t p = 0;; p += work_size) {
        while (j < ends.size() && ends[j] + j + 1 <= p) j++;
        if (j >= ends.size()) break;
        lr.push_back(crow[j]);
        ln.push_back(p - j);
    }
    ln.push_back(acc);
}

// MP_COL_PARTS upload: columns ranked by degree (as MP_COL_PERM), rank r in partition r % P at
// position base[r % P] + r / P of the gathered B (k_permute_rows); per partition its entries in
// row order (so every row's partial sums its entries in the plan's order), the merge-path wave
// ranges of that CSR, the in-launch combine state and (partitions >= 1) an fp32 output that
// k_add_parts adds to C in partition order (deterministic)
static void upload_col_parts(plan_state &p, device_arrays &a, const std::vector<uint64_t> &col,
                             const universal_array &vals) {
    device_plan &d = p.dev;
    const kernel_spec &sp = p.cg->get_kernel_spec();
    const meta_data_set &m = *p.meta;
    const int sb = p.cg->get_sub_matrix_id();
    const uint32_t P = d.mp_parts;
    const uint64_t K = p.K, nnz = col.size();
    const auto &rows = m.u(GLOBAL_META, "nz_row_indices", sb);
    const uint64_t row_num = row_num_of_sub_matrix(m, sb);
    std::vector<uint32_t> deg(K, 0u), perm(K), pos(K);
    for (uint64_t c : col) deg[c]++;
    for (uint32_t i = 0; i < (uint32_t)K; i++) perm[i] = i;
    std::stable_sort(perm.begin(), perm.end(), [&](uint32_t x, uint32_t y) { return deg[x] > deg[y]; });
    std::vector<uint64_t> base(P + 1, 0);
    // MP_HUB_COLS = H (P = 2): partition 0 = the H densest columns (the hubs, whose B rows stay in
    // the XCDs' L2s, so a round of that pass never waits on an Infinity-Cache / HBM gather),
    // partition 1 = the rest; else ranks are dealt round-robin over the P partitions
    const uint64_t hub = P == 2 ? (uint64_t)std::max<int64_t>(0, get_config().MP_HUB_COLS) : 0;
    if (hub > 0 && hub < K) {
        base[1] = hub;
        base[2] = K;
    } else {
        for (uint32_t x = 0; x < P; x++) base[x + 1] = base[x] + (K > x ? (K - x + P - 1) / P : 0);
    }
    std::vector<uint32_t> gather(K);
    for (uint32_t r = 0; r < (uint32_t)K; r++) {
        const uint32_t c = perm[r];
        const uint32_t q = hub > 0 && hub < K ? r : (uint32_t)(base[r % P] + r / P);
        pos[c] = q;
        gather[q] = c;
    }
    a.cperm = dev_copy(d, gather);
    const uint32_t Nd = (uint32_t)std::max<int64_t>(1, get_config().DENSE_MATRIX_SIZE);
    const size_t bb = (size_t)K * Nd * (d.dtype == 0 ? 4u : 2u);
    HIP_OK(hipMalloc(&a.bperm, std::max<size_t>(bb, 16)));
    d.allocations.push_back(a.bperm);
    const uint32_t cfv = d.dtype == 0 ? 4u : 8u, cf = Nd % cfv == 0 ? cfv : 1u;
    const uint32_t X = std::min<uint32_t>(64u, pow2ceil_u((Nd + cf - 1) / cf));
    const uint64_t target = (uint64_t)gsk::kMpItems * (64u / X);
    a.pp.assign((size_t)P * kMpPartPtrs, nullptr);
    d.mp_part_W.assign(P, 0);
    d.mp_part_rows.assign(P, 0);
    d.mp_part_fin.assign(P, 0);
    std::vector<uint8_t> part(nnz);
    std::vector<uint64_t> cnt(P, 0);
    for (uint64_t e = 0; e < nnz; e++) {
        const uint32_t q = pos[col[e]];
        uint32_t x = 0;
        while (q >= base[x + 1]) x++;
        part[e] = (uint8_t)x;
        cnt[x]++;
    }
    for (uint32_t x = 0; x < P; x++) {
        std::vector<uint64_t> rx;
        std::vector<uint32_t> cx;
        std::vector<float> vx;
        rx.reserve(cnt[x]);
        cx.reserve(cnt[x]);
        vx.reserve(cnt[x]);
        for (uint64_t e = 0; e < nnz; e++)
            if (part[e] == x) {
                rx.push_back(rows[e]);
                cx.push_back(pos[col[e]]);
                vx.push_back((float)vals.read_float_from_arr(e));
            }
        GS_CHECK(!rx.empty(), "MP_COL_PARTS: a column partition without entries (fewer columns than partitions?)");
        void **pp = &a.pp[(size_t)x * kMpPartPtrs];
        if (d.col_bytes == 2) {
            std::vector<uint16_t> c16(cx.begin(), cx.end());
            pp[MP_PART_COL] = dev_copy(d, c16, kPad);
        } else {
            pp[MP_PART_COL] = dev_copy(d, cx, kPad);
        }
        pp[MP_PART_VAL] = dev_copy(d, vx, kPad);
        std::vector<uint64_t> lr, ln;
        merge_path_levels(rx, row_num, (uint64_t)sp.work_size, lr, ln);
        gsk_host::merge_path_layout lay;
        std::string why;
        GS_CHECK(gsk_host::merge_path_device_layout(rx, row_num, lr, ln, (uint64_t)sp.work_size, (uint32_t)d.row_base, target,
                                                     lay, why, d.n_out_rows, 2 * target),
                 "merge-path layout of column partition " + std::to_string(x) + ": " + why);
        pp[MP_PART_WZ] = dev_copy(d, lay.wz);
        pp[MP_PART_WQ] = dev_copy(d, lay.wq);
        pp[MP_PART_ENDS] = dev_copy(d, lay.ends);
        pp[MP_PART_RID] = dev_copy(d, lay.rid);
        pp[MP_PART_EMPTY] = lay.empty.empty() ? nullptr : dev_copy(d, lay.empty);
        const uint32_t W = (uint32_t)(lay.wz.size() - 1);
        pp[MP_PART_WS] = dev_copy(d, std::vector<float>((size_t)W * Nd, 0.f));
        pp[MP_PART_WS2] = dev_copy(d, std::vector<float>((size_t)W * Nd, 0.f));
        pp[MP_PART_T0] = dev_copy(d, std::vector<uint32_t>(W, 0xffffffffu));
        pp[MP_PART_CHAIN] = dev_copy(d, lay.chain);
        pp[MP_PART_CNT] = dev_copy(d, std::vector<uint32_t>(W, 0u));
        if (x > 0) pp[MP_PART_OUT] = dev_copy(d, std::vector<float>((size_t)d.n_out_rows * Nd, 0.f));
        d.mp_part_W[x] = W;
        d.mp_part_rows[x] = (uint32_t)lay.ends.size();
        d.mp_part_fin[x] = (uint32_t)lay.empty.size();
    }
    // the whole-matrix CSR is not uploaded: part 0's columns stand in for it (non-null)
    a.col = a.pp[MP_PART_COL];
    a.val = a.pp[MP_PART_VAL];
}

// the plan's column indices (u16 when they fit, else u32) and values (plan dtype) of
// one replica, padded for the kernels' aligned over-reads
void upload_csr(plan_state &p, device_arrays &a) {
    const kernel_spec &sp = p.cg->get_kernel_spec();
    const meta_data_set &m = *p.meta;
    const int sb = p.cg->get_sub_matrix_id();
    device_plan &d = p.dev;
    HIP_OK(hipSetDevice(d.device));
    const auto &col = m.u(GLOBAL_META, sp.interleaved ? "nz_col_indices_after_interlance_storage" : "nz_col_indices", sb);
    auto vals = m.get_element(GLOBAL_META, sp.interleaved ? "nz_vals_after_interlance_storage" : "nz_vals", sb)->meta_data_arr;
    const uint64_t nnz = col.size();
    if (d.mp_parts > 1) {
        upload_col_parts(p, a, col, *vals);
        return;
    }
    if (d.col_perm) {
        // MP_COL_PERM: columns renumbered by degree (most nonzeros first, ties by column), so
        // the B rows the power-law hubs gather share 128-B lines and stay in L2; each launch
        // first gathers B into that order (k_permute_rows).  Only the device copy of the
        // column indices changes; the order of every row's entries, so every sum, is the same
        std::vector<uint32_t> deg(p.K, 0u), perm(p.K), rank(p.K);
        for (uint64_t c : col) deg[c]++;
        for (uint32_t i = 0; i < (uint32_t)p.K; i++) perm[i] = i;
        const uint64_t hot = (uint64_t)std::max<int64_t>(0, get_config().MP_PERM_HOT);
        if (hot == 0 || hot >= p.K) {
            std::stable_sort(perm.begin(), perm.end(), [&](uint32_t x, uint32_t y) { return deg[x] > deg[y]; });
        } else {  // MP_PERM_HOT: the `hot` densest columns first (by degree), the rest in their own order
            std::vector<uint32_t> byd(perm);
            std::nth_element(byd.begin(), byd.begin() + hot, byd.end(), [&](uint32_t x, uint32_t y) {
                return deg[x] != deg[y] ? deg[x] > deg[y] : x < y;
            });
            byd.resize(hot);
            std::sort(byd.begin(), byd.end(), [&](uint32_t x, uint32_t y) { return deg[x] != deg[y] ? deg[x] > deg[y] : x < y; });
            std::vector<uint8_t> is_hot(p.K, 0);
            for (uint32_t c : byd) is_hot[c] = 1;
            size_t w = 0;
            for (uint32_t c : byd) perm[w++] = c;
            for (uint32_t c = 0; c < (uint32_t)p.K; c++)
                if (!is_hot[c]) perm[w++] = c;
        }
        for (uint32_t i = 0; i < (uint32_t)p.K; i++) rank[perm[i]] = i;
        std::vector<uint32_t> c32(nnz);
        for (uint64_t i = 0; i < nnz; i++) c32[i] = rank[col[i]];
        if (d.col_bytes == 2) {
            std::vector<uint16_t> c16(c32.begin(), c32.end());
            a.col = dev_copy(d, c16, kPad);
        } else {
            a.col = dev_copy(d, c32, kPad);
        }
        d.perm_scatter = get_config().MP_PERM_SCATTER != 0;
        a.cperm = dev_copy(d, d.perm_scatter ? rank : perm);  // scatter: new place of each column
        // the gathered B: K rows of the plan's dense width (launches check N <= ws_n = that width)
        const size_t bb = (size_t)p.K * (size_t)std::max<int64_t>(1, get_config().DENSE_MATRIX_SIZE) * (d.dtype == 0 ? 4u : 2u);
        HIP_OK(hipMalloc(&a.bperm, std::max<size_t>(bb, 16)));
        d.allocations.push_back(a.bperm);
    } else if (d.col_bytes == 2) {
        std::vector<uint16_t> c16(col.begin(), col.end());
        a.col = dev_copy(d, c16, kPad);
    } else {
        a.col = dev_copy(d, to_u32(col, "column index"), kPad);
    }
    if (d.dtype == 0) {
        std::vector<float> v(nnz);
        for (uint64_t i = 0; i < nnz; i++) v[i] = (float)vals->read_float_from_arr(i);
        a.val = dev_copy(d, v, kPad);
    } else {
        std::vector<uint16_t> v(nnz);
        for (uint64_t i = 0; i < nnz; i++) v[i] = f32_to_f16_bits((float)vals->read_float_from_arr(i));
        a.val = dev_copy(d, v, kPad);
    }
}

void upload_plan(plan_state &p, int dtype, int device) {
    GS_CHECK(p.cg && p.cg->is_compiled(), "plan must be compiled before upload");
    GS_CHECK(dtype == 0 || dtype == 1, "dtype must be 0 (fp32) or 1 (fp16)");
    free_device(p);
    HIP_OK(hipSetDevice(device));
    const kernel_spec &sp = p.cg->get_kernel_spec();
    const meta_data_set &m = *p.meta;
    const int sb = p.cg->get_sub_matrix_id();
    device_plan &d = p.dev;
    d = device_plan();
    d.device = device;
    d.dtype = dtype;
    // a parent-indexed sub-matrix (row_nz_matrix_div_operator) writes a scratch output whose
    // row r is its row index r (capi.cc combines the scratch outputs into C)
    const bool pidx = p.parent_row_base >= 0;
    d.row_base = pidx ? 0 : m.scalar(GLOBAL_META, "begin_row_index", sb);
    // output rows this plan writes: all of C for the undivided matrix; a sub-matrix of a
    // row division (§8f rank 3) owns [begin_row_index, begin_row_index + its rows) only
    const uint64_t out_lo = sb == 0 || pidx ? 0 : d.row_base;
    const uint64_t out_hi = sb == 0 ? p.M : d.row_base + row_num_of_sub_matrix(m, sb);
    d.n_out_rows = out_hi;
    d.out_lo = out_lo;
    const auto &rows = m.u(GLOBAL_META, "nz_row_indices", sb);
    // interleaved storage (§8f rank 2): the kernel streams the permuted arrays
    const auto &col = m.u(GLOBAL_META, sp.interleaved ? "nz_col_indices_after_interlance_storage" : "nz_col_indices", sb);
    auto vals = m.get_element(GLOBAL_META, sp.interleaved ? "nz_vals_after_interlance_storage" : "nz_vals", sb)->meta_data_arr;
    if (sp.interleaved && sp.interleave_parent == GLOBAL_META)
        d.ilv = (uint32_t)m.u(GLOBAL_META, "BMT_size_of_each_blk", sb).at(0);
    uint64_t nnz = col.size();
    GS_CHECK(nnz < 0xffffffffull - kPad, "nnz exceeds 32-bit offsets");
    d.nnz_stored = nnz;
    device_arrays a;
    // the matrix-core layout (device_layout.cc: the same choice the emitted program makes)
    mc_layout mc = choose_matrix_core_layout(m, sp, sb, p.K, dtype);
    if (mc.kind == mc_layout::NM) {
        // col-direction BMTs that are 2:4 panels: sparse matrix cores, self-contained blocks
        d.nm = true;
        d.kernel = mc.nm_ks ? "k_nm_mfma_ks" : (mc.nm4 ? "k_nm_mfma4" : "k_nm_mfma");
        d.nm4 = mc.nm4;
        d.nm_nt = mc.nm_nt;
        d.nm_tiles = mc.nm_T;
        d.KC = mc.nm_S;
        d.n_rows_aux = mc.nm_rows;
        d.n_units = m.u(THREAD_META, "first_nz_indices", sb).size() - 1;
        d.waves = mc.nm_ks ? 4 : gsk::kNmWaves;
        d.nm_ks = mc.nm_ks;
        d.ksplit = mc.nm_ks || mc.nm4 ? mc.nm_split : 1;
        d.ncs = mc.nm_ncs;
        a.tcol = dev_copy(d, mc.nm_blk);
        d.bytes_tile = d.bytes_A;
        if (mc.nm_ks && mc.nm_split > 1) {  // fp32 slabs (one 64 x N tile per row group and K range) + counters
            const uint64_t ngr = (mc.nm_rows + 255) / 256 * 4;
            a.ws = dev_copy(d, std::vector<float>((size_t)ngr * mc.nm_split * 64 * mc.N, 0.f));
            a.t2 = dev_copy(d, std::vector<uint32_t>((size_t)ngr, 0u));
        }
        if (mc.nm4 && mc.nm_split > 1) {  // tagged fp32 slabs (256 x N per unit), counters + the device error word
            const uint64_t nb = (mc.nm_rows + 255) / 256;
            a.ws = dev_copy(d, std::vector<float>((size_t)nb * mc.nm_split * 256 * mc.N, 0.f));
            a.t2 = dev_copy(d, std::vector<uint32_t>((size_t)nb + 1u, 0u));
            d.err_at = nb;
        }
        d.replicas.push_back(a);
        p.uploaded = true;
        return;
    }
    // A streams: narrowest column type that holds Kc-1 (u16 when Kc <= 65536).  fp16 BMTB
    // plans try the matrix cores first: their kernels never read the CSR arrays, which
    // are then uploaded only if a launch at another dense width falls back to a gather
    // kernel (ensure_csr), so A is not resident twice.
    uint64_t maxc = 0;
    for (uint64_t c : col) maxc = std::max(maxc, c);
    d.col_bytes = maxc <= 0xffff ? 2 : 4;
    const bool defer_csr = dtype == 1 && get_config().MFMA_TILES &&
                           (sp.family == KF_WARP_TOTAL || sp.family == KF_BLOCK_TOTAL) &&
                           m.is_exist(TBLOCK_META, "first_row_indices", sb);
    if (sp.family == KF_MERGE_PATH) {
        // MP_COL_PERM (decided before the CSR upload, which renumbers the columns)
        const config_t cfg = get_config();
        const uint64_t b_bytes = p.K * (uint64_t)std::max<int64_t>(1, cfg.DENSE_MATRIX_SIZE) * (dtype == 0 ? 4u : 2u);
        d.col_perm = !sp.interleaved && p.K < (1ull << 32) &&
                     (cfg.MP_COL_PERM > 0 || (cfg.MP_COL_PERM < 0 && b_bytes >= (64ull << 20)));
        // MP_COL_PARTS (fp32 plans of the whole matrix, one column tile: N <= 32): the renumbered
        // columns dealt over P partitions, one merge-path pass each (upload_col_parts)
        const int64_t Nd = std::max<int64_t>(1, cfg.DENSE_MATRIX_SIZE);
        if (d.col_perm && dtype == 0 && sb == 0 && !pidx && cfg.MP_COL_PARTS > 1 && Nd <= 32 && p.K >= 64 * (uint64_t)cfg.MP_COL_PARTS)
            d.mp_parts = (uint32_t)std::min<int64_t>(cfg.MP_COL_PARTS, 8);
    }
    if (!defer_csr) upload_csr(p, a);
    GS_CHECK(!d.col_perm || (a.cperm && a.bperm), "merge-path column permutation: arrays not uploaded");
    uint64_t row_num = row_num_of_sub_matrix(m, sb);
    // matrix-core row blocks for fp16 plans with BMTBs (tried before the other kernels)
    auto try_mfma = [&](const std::vector<uint32_t> &) {
        if (mc.kind == mc_layout::KS) {
            // tall row blocks: K split over workgroups, wave-autonomous (k_mfma_ks)
            const ks_tiles &kt = mc.ks;
            d.mfma = true;
            d.ks = true;
            d.kernel = "k_mfma_ks";
            d.lds_N = mc.N;
            d.ksplit = kt.S;
            d.ks_ns = kt.NS;
            d.maxr = kt.RT;
            d.rpw_max = kt.RMAX;
            d.seg_cap = kt.MAXG;
            d.waves = kt.W;
            d.lds_bytes = kt.lds_bytes;
            const uint64_t nb = mc.tbr.size() - 1;
            d.n_rows_aux = nb;
            const size_t before = d.bytes_A;
            d.ks_gcap = kt.GCAP;
            d.ks_ctw = kt.CT;
            d.ks_ap = kt.AP;
            d.ks_p8 = kt.P8;
            d.ks_nt = kt.NT;
            d.ks_gh = kt.GH;
            d.ks_persist = (uint32_t)std::max<int64_t>(0, get_config().KS_PERSIST);
            if (d.ks_persist) a.t3 = dev_copy(d, std::vector<uint32_t>(9, 0u));  // 8 XCD heads + the exit count
            a.t0 = dev_copy(d, to_u32(mc.tbr, "BMTB first_row_indices"));
            a.tcol = kt.P8 ? (void *)dev_copy(d, kt.pos8) : (void *)dev_copy(d, kt.pos);
            a.tval = dev_copy(d, kt.val);
            a.t1 = dev_copy(d, kt.steps);
            d.bytes_tile = d.bytes_A - before;
            if (kt.S > 1) {
                const uint32_t CT = kt.CT, nt = ks_col_tiles_ct(mc.N, CT);
                a.ws = dev_copy(d, std::vector<float>((size_t)nb * kt.S * nt * 256 * kt.RT * CT, 0.f));
                // arrival counters, then the replica's device error word (ks_slab_wait)
                a.t2 = dev_copy(d, std::vector<uint32_t>((size_t)nb * nt + 1u, 0u));
                d.err_at = (uint64_t)nb * nt;
            }
            return true;
        }
        if (mc.kind == mc_layout::BM) {
            // bitmap records, fragments expanded in registers (k_mfma_bm)
            const bm_tiles &bt = mc.bm;
            d.mfma = true;
            d.bm = true;
            d.bm2 = bt.v2;
            d.bmkb = bt.kb;
            d.seg_cap = bt.NVB;  // k_mfma_kb: KB of values per k-step
            d.kernel = bt.kb ? "k_mfma_kb" : bt.v2 ? "k_mfma_bm2" : "k_mfma_bm";
            d.lds_N = mc.N;
            d.ksplit = bt.S;
            d.ks_ns = bt.NS;
            d.maxr = bt.RT;
            d.rpw_max = bt.RMAX;
            d.waves = bt.W;
            d.lds_bytes = bt.lds_bytes;
            const uint64_t nb = mc.tbr.size() - 1;
            d.n_rows_aux = nb;
            const size_t before = d.bytes_A;
            a.t0 = dev_copy(d, to_u32(mc.tbr, "BMTB first_row_indices"));
            a.tcol = dev_copy(d, bt.rec);
            a.t1 = dev_copy(d, bt.sbase);
            a.tval = dev_copy(d, bt.val);
            d.bytes_tile = d.bytes_A - before;
            if (bt.S > 1) {
                const uint32_t nt = ks_col_tiles(mc.N), CT = ks_ct(mc.N);
                a.ws = dev_copy(d, std::vector<float>((size_t)nb * bt.S * nt * 256 * bt.RT * CT, 0.f));
                // arrival counters: per (row block, column tile), per row tile too for k_mfma_bm2
                a.t2 = dev_copy(d, std::vector<uint32_t>((size_t)nb * nt * (bt.v2 ? bt.RT : 1u) + 1u, 0u));
                if (bt.kb) d.err_at = (uint64_t)nb * nt;  // k_mfma_kb: the device error word after the counters
            }
            return true;
        }
        if (mc.kind != mc_layout::ROWS) return false;
        const mfma_tiles &t = mc.rows;
        d.mfma = true;
        d.kernel = "k_mfma_rows";
        d.lds_N = mc.N;
        d.KC = 1u << t.lgKC; d.nc = t.nc; d.maxr = t.RT; d.rpw_max = t.RMAX; d.RSB = t.lgKC;
        d.seg_cap = t.gmax;
        d.mfma_glds = mc.rows_glds; d.mfma_nbg = mc.rows_nbg; d.mfma_wct = mc.rows_wct; d.mfma_maxa = mc.rows_maxa;
        d.mfma_flags = mc.rows_flags;
        const uint64_t nb = mc.tbr.size() - 1;
        d.ncs = mc.rows_ncs;
        d.ksplit = mc.rows_ksplit;
        if (d.ksplit > 1) {
            std::vector<float> z((size_t)nb * d.ksplit * t.RMAX * mc.N, 0.f);
            a.ws = dev_copy(d, z);
            a.t2 = dev_copy(d, std::vector<uint32_t>(nb, 0u));  // arrival counters
        }
        d.waves = kMfmaThreads / 64; d.lds_bytes = t.lds_bytes;
        const size_t before = d.bytes_A;
        a.t0 = dev_copy(d, to_u32(mc.tbr, "BMTB first_row_indices"));
        a.t1 = dev_copy(d, t.seg_start);
        a.tcol = dev_copy(d, t.pos);
        a.tval = dev_copy(d, t.val);
        d.bytes_tile = d.bytes_A - before;
        d.n_rows_aux = nb;
        return true;
    };
    switch (sp.family) {
        case KF_THREAD_TOTAL: {
            const auto &fn = m.u(THREAD_META, "first_nz_indices", sb);
            const auto &fr = m.u(THREAD_META, "first_row_indices", sb);
            for (size_t i = 0; i < fr.size(); i++)
                GS_CHECK(fr[i] == i, "thread_total kernel needs one row per BMT (fixed_row_block_size 1)");
            bool al4 = true, al8 = true;
            for (uint64_t x : fn) { al4 &= (x % 4 == 0); al8 &= (x % 8 == 0); }
            d.scf = al8 ? 8 : (al4 ? 4 : 1);
            a.a0 = upload_index(d, m, THREAD_META, "first_nz_indices", sb, d.f0);
            if (m.is_exist(GLOBAL_META, "original_nz_row_indices", sb)) {
                a.a1 = upload_index(d, m, GLOBAL_META, "original_nz_row_indices", sb, d.f1);
                d.n_rows_aux = m.u(GLOBAL_META, "original_nz_row_indices", sb).size();
            } else {
                // rows were not sorted: the row of BMT i is i (the reference indexes C by it
                // directly); an identity array unless the formulas are on
                std::vector<uint64_t> order(row_num);
                for (uint64_t r = 0; r < row_num; r++) order[r] = r;
                a.a1 = upload_index(d, order, UNSIGNED_INT, "row order", d.f1);
                d.n_rows_aux = row_num;
            }
            d.n_units = fn.size() - 1;
            break;
        }
        case KF_WARP_TOTAL: {
            // BMW rows and BMTB->BMW map: formulas for k_warp_rows; k_lds_rows reads the arrays
            auto upload_groups = [&](bool formulas) {
                if (formulas) {
                    a.a0 = upload_index(d, m, sp.group_level, "first_row_indices", sb, d.f0);
                    if (sp.tblock_parent) a.a1 = upload_index(d, m, TBLOCK_META, "first_BMW_indices", sb, d.f1);
                } else {
                    a.a0 = dev_copy(d, to_u32(m.u(sp.group_level, "first_row_indices", sb), "BMW first_row_indices"));
                    if (sp.tblock_parent)
                        a.a1 = dev_copy(d, to_u32(m.u(TBLOCK_META, "first_BMW_indices", sb), "first_BMW_indices"));
                }
            };
            if (sp.tblock_parent) d.n_rows_aux = m.u(TBLOCK_META, "first_BMW_indices", sb).size() - 1;  // BMTB count
            std::vector<uint32_t> rp = csr_row_ptr(rows, row_num);
            a.a2 = dev_copy(d, rp);
            d.n_units = m.u(sp.group_level, "first_row_indices", sb).size() - 1;
            {
                const auto &gr = m.u(sp.group_level, "first_row_indices", sb);
                uint64_t mx = 0;
                for (size_t i = 0; i + 1 < gr.size(); i++) mx = std::max<uint64_t>(mx, gr[i + 1] - gr[i]);
                d.bmw_rows_max = (uint32_t)mx;
                d.mean_row_nnz = row_num ? (double)rp.back() / (double)row_num : 0.0;
            }
            d.scf = 4;
            if (sp.tblock_parent && try_mfma(rp)) {
                upload_groups(true);  // the gather fallback at other dense widths
                break;
            }
            // LDS-stationary B pays off for row blocks of >= 16 rows in BMWs of >= 2 rows
            // (C2: 20x2 31 us vs 40 us gathered; 4x1 62 us): otherwise the gather kernel
            bool lds_worth = false;
            if (sp.tblock_parent) {
                const auto &tr = m.u(TBLOCK_META, "first_row_indices", sb);
                const auto &wr = m.u(WARP_META, "first_row_indices", sb);
                uint64_t mt = 0, mw = 0;
                for (size_t i = 0; i + 1 < tr.size(); i++) mt = std::max<uint64_t>(mt, tr[i + 1] - tr[i]);
                for (size_t i = 0; i + 1 < wr.size(); i++) mw = std::max<uint64_t>(mw, wr[i + 1] - wr[i]);
                lds_worth = mt >= 16 && mw >= 2;
            }
            if (sp.tblock_parent && get_config().LDS_STAGE_B && lds_worth) {
                lds_tiles t;
                std::string why;
                const uint32_t Nd = (uint32_t)get_config().DENSE_MATRIX_SIZE;
                size_t budget = (size_t)std::min<int64_t>(get_config().SHARED_MEM_TOTAL_SIZE, 160 * 1024);
                // LDS_DMA (fp32 at N = 32): chunks by LDS-DMA into two buffers (k_lds_rows_dma), at most
                // 80 KB per workgroup so two share a CU (their barriers and DMA waits interleave; the auto
                // K split below makes the grid two per CU): C2 fp32 (20,2) 37.7 -> 34.4 us (r06r)
                const bool dma = dtype == 0 && Nd == 32 && get_config().LDS_DMA != 0;
                if (dma) budget = std::min<size_t>(budget, 80 * 1024);
                // LDS_KSPLIT: S workgroups per BMTB, each over ncs consecutive chunks of K
                // (every K range non-empty), fp32 slabs + one arrival counter per BMTB.  0 (auto):
                // plans of under 128 BMTBs split K until ~256 workgroups (a workgroup's time
                // is its nonzeros: C2 fp32 (20,2) 41.5 us = (40,4) in 2 K ranges 44.5 us,
                // profiles/r06f_lds_ksplit.txt, so full grids gain nothing from a split)
                // With LDS-DMA (two workgroups per CU) the auto split aims at ~512 workgroups.
                const uint64_t nbt0 = m.u(TBLOCK_META, "first_row_indices", sb).size() - 1;
                const int64_t cfg_ks = get_config().LDS_KSPLIT;
                const uint64_t wg_aim = dma ? 512 : 256;
                const uint32_t want = cfg_ks > 0 ? (uint32_t)cfg_ks
                                                 : (nbt0 * 2 <= wg_aim ? (uint32_t)std::max<uint64_t>(1, wg_aim / std::max<uint64_t>(nbt0, 1)) : 1u);
                if (build_lds_tiles(m.u(TBLOCK_META, "first_row_indices", sb), m.u(TBLOCK_META, "first_BMW_indices", sb),
                                    m.u(WARP_META, "first_row_indices", sb), rp, col, p.K, Nd, dtype ? 2u : 4u, budget,
                                    t, why, dma, want)) {
                    d.lds = true;
                    d.lds_dma = dma;
                    d.kernel = t.maxr == 8 ? "k_lds_rows_rs" : (dma ? "k_lds_rows_dma" : "k_lds_rows");
                    const uint32_t ncs = (t.nc + std::min(want, t.nc) - 1) / std::min(want, t.nc);
                    d.ksplit = (t.nc + ncs - 1) / ncs;
                    d.ncs = ncs;
                    d.lds_N = Nd;
                    d.KC = t.KC; d.nc = t.nc; d.RSB = t.RSB; d.rpw_max = t.rpw_max; d.seg_cap = t.seg_cap;
                    d.waves = t.waves; d.maxr = t.maxr; d.lds_bytes = t.lds_bytes;
                    const size_t before = d.bytes_A;
                    a.t0 = dev_copy(d, to_u32(m.u(TBLOCK_META, "first_row_indices", sb), "BMTB first_row_indices"));
                    a.t1 = dev_copy(d, t.seg_start);
                    a.t2 = dev_copy(d, t.seg_row_off);
                    a.tcol = dev_copy(d, t.tcol, kPad);
                    if (dtype == 0) {
                        std::vector<float> v(t.src.size());
                        for (size_t i = 0; i < v.size(); i++)
                            v[i] = t.src[i] == ~0u ? 0.f : (float)vals->read_float_from_arr(t.src[i]);
                        a.tval = dev_copy(d, v, kPad);
                    } else {
                        std::vector<uint16_t> v(t.src.size());
                        for (size_t i = 0; i < v.size(); i++)
                            v[i] = t.src[i] == ~0u ? 0 : f32_to_f16_bits((float)vals->read_float_from_arr(t.src[i]));
                        a.tval = dev_copy(d, v, kPad);
                    }
                    d.bytes_tile = d.bytes_A - before;
                    if (d.ksplit > 1) {
                        const uint64_t nbt = m.u(TBLOCK_META, "first_row_indices", sb).size() - 1;
                        a.ws = dev_copy(d, std::vector<float>((size_t)nbt * d.ksplit * t.rpw_max * Nd, 0.f));
                        a.t3 = dev_copy(d, std::vector<uint32_t>((size_t)nbt, 0u));
                    }
                }
            }
            upload_groups(!d.lds);
            break;
        }
        case KF_BLOCK_TOTAL: {
            a.a0 = upload_index(d, m, TBLOCK_META, "first_row_indices", sb, d.f0);
            std::vector<uint32_t> rp = csr_row_ptr(rows, row_num);
            a.a2 = dev_copy(d, rp);
            d.n_units = m.u(TBLOCK_META, "first_row_indices", sb).size() - 1;
            d.scf = 4;
            try_mfma(rp);
            break;
        }
        case KF_BITMAP_SEGMENT: {
            const auto &fn = m.u(THREAD_META, "first_nz_indices", sb);
            uint64_t nb = fn.size() - 1;
            for (uint64_t i = 0; i < nb; i++) {
                GS_CHECK(fn[i + 1] - fn[i] <= 64, "bitmap kernel needs BMTs of at most 64 nnz");
                GS_CHECK(fn[i] % 8 == 0, "bitmap kernel needs 8-aligned BMTs");
            }
            // real row starts (the plan's thread_bit_map also carries the forced BMW heads)
            std::vector<uint64_t> mask(nb, 0);
            for (uint64_t i = 0; i < nb; i++) {
                uint64_t mm = 0;
                for (uint64_t j = fn[i]; j < fn[i + 1]; j++)
                    if (j == 0 || rows[j] != rows[j - 1]) mm |= 1ull << (j - fn[i]);
                mask[i] = mm;
            }
            a.a0 = upload_index(d, m, THREAD_META, "first_nz_indices", sb, d.f0);
            a.a1 = upload_index(d, m, THREAD_META, "first_row_indices", sb, d.f1);
            a.m0 = dev_copy(d, mask);
            a.a2 = dev_copy(d, to_u32(m.u(THREAD_META, "segment_ptr", sb), "segment_ptr"));
            a.a3 = dev_copy(d, to_u32(m.u(THREAD_META, "segment_empty_row_indices", sb), "segment_empty_row_indices"));
            d.n_units = nb;
            d.scf = 4;
            if (dtype == 1) {
                // fp16 C: rows whose nonzeros span BMTs accumulate in an fp32 workspace and
                // are rounded once by k_finalize_rows, which also writes the empty rows (no memset)
                const uint64_t rb = d.row_base;
                std::vector<uint32_t> rp = csr_row_ptr(rows, row_num);
                std::vector<uint8_t> fin(p.M, 0);
                for (uint64_t r = out_lo; r < out_hi; r++)
                    if (r < rb || r - rb >= row_num || rp[r - rb] == rp[r - rb + 1]) fin[r] = 1;
                for (uint64_t i = 1; i + 1 < fn.size(); i++) {  // a BMT boundary strictly inside a row
                    const uint64_t z = fn[i];
                    if (z == 0 || z >= rows.size()) continue;
                    if (rows[z] == rows[z - 1]) fin[rows[z] + rb] = 1;
                }
                std::vector<uint32_t> list;
                for (uint64_t r = 0; r < p.M; r++)
                    if (fin[r]) list.push_back((uint32_t)r);
                a.a4 = dev_copy(d, list);
                a.ws = dev_copy(d, std::vector<float>((size_t)p.M * std::max<uint32_t>(1, (uint32_t)get_config().DENSE_MATRIX_SIZE), 0.f));
                d.ws_n = (uint32_t)get_config().DENSE_MATRIX_SIZE;
                d.n_fin = list.size();
            } else {
                d.needs_memset = true;
            }
            break;
        }
        case KF_ROW_CHUNKS: {
            // chunks of one row: col-direction BMTs, or col-direction BMWs / BMTBs (the spec's
            // first array names the level)
            const POS_TYPE L = sp.arrays[0].rfind("WARP_META", 0) == 0
                                   ? WARP_META
                                   : (sp.arrays[0].rfind("TBLOCK_META", 0) == 0 ? TBLOCK_META : THREAD_META);
            const auto &fn = m.u(L, "first_nz_indices", sb);
            const auto &fr = m.u(L, "first_row_indices_without_ending", sb);
            GS_CHECK(fn.size() == fr.size() + 1 && !fr.empty(), "col-direction plan: chunk arrays disagree");
            std::vector<uint32_t> br = to_u32(fr, "first_row_indices_without_ending");
            a.a0 = upload_index(d, m, L, "first_nz_indices", sb, d.f0);
            a.a1 = upload_index(d, m, L, "first_row_indices_without_ending", sb, d.f1);
            d.n_units = br.size();
            d.scf = 4;
            d.span = gsk_host::row_chunk_span(br.size());
            if (sp.interleaved && sp.interleave_parent != GLOBAL_META) {
                // per-parent interleaving: BMT b of parent j (first BMT F, first nonzero P, n BMTs)
                // has its i-th nonzero at P + (b - F) + i * n (k_row_chunks ilv_base / ilv_stride)
                const POS_TYPE pp = (POS_TYPE)sp.interleave_parent;
                const auto &pf = m.u(pp, "first_BMT_indices", sb);
                const auto &pn = m.u(pp, "first_nz_indices", sb);
                GS_CHECK(pf.size() == pn.size() && !pf.empty() && pf.back() == br.size(),
                         "interleaved parents: first_BMT_indices / first_nz_indices disagree with the BMTs");
                std::vector<uint32_t> ib(br.size()), is(br.size());
                for (size_t j = 0; j + 1 < pf.size(); j++)
                    for (uint64_t b = pf[j]; b < pf[j + 1]; b++) {
                        ib[b] = (uint32_t)(pn[j] + (b - pf[j]));
                        is[b] = (uint32_t)(pf[j + 1] - pf[j]);
                    }
                a.a2 = dev_copy(d, ib);
                a.a3 = dev_copy(d, is);
            }
            // rows shared by two waves' BMT ranges accumulate in an fp32 workspace; the
            // finalize pass rounds them and writes the rows without BMTs (no memset)
            std::vector<uint32_t> list = gsk_host::row_chunk_finalize_rows(br, p.M, d.span, (uint32_t)d.row_base);
            list.erase(std::remove_if(list.begin(), list.end(), [&](uint32_t r) { return r < out_lo || r >= out_hi; }),
                       list.end());
            d.ws_n = (uint32_t)std::max<int64_t>(1, get_config().DENSE_MATRIX_SIZE);
            a.ws = dev_copy(d, std::vector<float>((size_t)p.M * d.ws_n, 0.f));
            if (!list.empty()) a.a4 = dev_copy(d, list);
            d.n_fin = list.size();
            break;
        }
        case KF_MERGE_PATH: {
            // wave ranges decoded from the merge-path levels; S = 64/X slots per wave as launched
            const POS_TYPE L = sp.merge_level;
            const uint32_t Nd = (uint32_t)std::max<int64_t>(1, get_config().DENSE_MATRIX_SIZE);
            const uint32_t cfv = dtype == 0 ? 4u : 8u, cf = Nd % cfv == 0 ? cfv : 1u;
            const uint32_t X = std::min<uint32_t>(64u, pow2ceil_u((Nd + cf - 1) / cf));
            const uint64_t target = (uint64_t)gsk::kMpItems * (64u / X);  // >= one round per wave
            if (d.mp_parts > 1) {  // the partitions' layouts are built with their CSRs (upload_col_parts)
                d.scf = 8;
                d.ws_n = Nd;
                d.n_units = d.mp_part_W[0];
                d.kernel = "k_merge_path";
                break;
            }
            gsk_host::merge_path_layout lay;
            std::string why;
            GS_CHECK(gsk_host::merge_path_device_layout(rows, row_num, m.u(L, "first_row_indices_without_ending", sb),
                                                         m.u(L, "first_nz_indices", sb), (uint64_t)sp.work_size,
                                                         (uint32_t)d.row_base, target, lay, why, d.n_out_rows,
                                                         2 * target),
                     "merge-path layout: " + why);
            a.a0 = dev_copy(d, lay.wz);
            a.a1 = dev_copy(d, lay.wq);
            a.a2 = dev_copy(d, lay.ends);
            a.a3 = dev_copy(d, lay.rid);
            a.a4 = dev_copy(d, lay.empty);
            d.n_fin = lay.empty.size();
            d.n_units = lay.wz.size() - 1;
            d.n_rows_aux = lay.ends.size();
            d.ws_n = Nd;
            a.ws = dev_copy(d, std::vector<float>((size_t)d.n_units * Nd, 0.f));
            a.ws2 = dev_copy(d, std::vector<float>((size_t)d.n_units * Nd, 0.f));
            a.t0 = dev_copy(d, std::vector<uint32_t>(d.n_units, 0xffffffffu));
            a.t1 = dev_copy(d, lay.chain);                                 // split-row chains
            a.t2 = dev_copy(d, std::vector<uint32_t>(d.n_units, 0u));     // their arrival counters
            d.scf = 8;
            {
                const config_t cfg = get_config();
                d.mp_rows = cfg.MP_ROWS;
                d.mp_solo = (uint32_t)std::max<int64_t>(1, cfg.MP_SOLO);
                d.kernel = d.mp_rows ? "k_merge_rows" : "k_merge_path";
            }
            break;
        }
        default:
            throw gs_error("no gfx950 kernel family for this plan");
    }
    if (defer_csr && !d.mfma) upload_csr(p, a);
    // row-padded plans (modify_*_by_row_pad_in_sub_matrix): the padding rows lie past the
    // output, so every launch writes a scratch output of all the plan's rows and launch_spmm
    // copies its first M rows to C
    const uint64_t prows = row_num_of_sub_matrix(m, sb);
    if (sb == 0 && !pidx && prows > p.M) {
        d.pad_rows = prows;
        d.pad_N = (uint32_t)std::max<int64_t>(1, get_config().DENSE_MATRIX_SIZE);
        a.pad_out = dev_copy(d, std::vector<uint32_t>((prows * d.pad_N * (dtype == 0 ? 4u : 2u) + 3) / 4, 0u));
    }
    d.replicas.push_back(a);
    p.uploaded = true;
}

// The deferred CSR of a matrix-core plan, uploaded the first time the plan runs at a dense
// width other than the one its tiles were built for.  Synchronous (hipMalloc + hipMemcpy),
// so refused inside stream capture (launch_body); the caller's current device is restored.
void ensure_csr(plan_state &p) {
    bool need = false;
    for (device_arrays &a : p.dev.replicas) need |= !a.col;
    if (!need) return;
    int prev = 0;
    HIP_OK(hipGetDevice(&prev));
    for (device_arrays &a : p.dev.replicas)
        if (!a.col) upload_csr(p, a);
    HIP_OK(hipSetDevice(prev));
}

void add_replica(plan_state &p) {
    GS_CHECK(p.uploaded, "upload the plan before adding replicas");
    HIP_OK(hipSetDevice(p.dev.device));
    const device_arrays &s = p.dev.replicas[0];
    device_arrays r = s;
    // every allocation of replica 0 is duplicated (same sizes)
    size_t n0 = p.dev.allocations.size();
    std::vector<void *> base(p.dev.allocations.begin(), p.dev.allocations.begin() + n0);
    auto dup = [&](void *src) -> void * {
        if (!src) return nullptr;
        size_t bytes = 0;
        HIP_OK(hipMemPtrGetInfo(src, &bytes));
        void *dst = nullptr;
        HIP_OK(hipMalloc(&dst, bytes));
        HIP_OK(hipMemcpy(dst, src, bytes, hipMemcpyDeviceToDevice));
        p.dev.allocations.push_back(dst);
        return dst;
    };
    r.col = s.pp.empty() ? dup(s.col) : nullptr;  // MP_COL_PARTS: stand-ins for part 0 (below)
    r.val = s.pp.empty() ? dup(s.val) : nullptr;
    r.a0 = (uint32_t *)dup(s.a0);
    r.a1 = (uint32_t *)dup(s.a1);
    r.a2 = (uint32_t *)dup(s.a2);
    r.a3 = (uint32_t *)dup(s.a3);
    r.a4 = (uint32_t *)dup(s.a4);
    r.m0 = (uint64_t *)dup(s.m0);
    r.tcol = dup(s.tcol);
    r.tval = dup(s.tval);
    r.t0 = (uint32_t *)dup(s.t0);
    r.t1 = (uint32_t *)dup(s.t1);
    r.t2 = (uint32_t *)dup(s.t2);
    r.t3 = (uint32_t *)dup(s.t3);
    r.t4 = (uint32_t *)dup(s.t4);
    r.ws = (float *)dup(s.ws);
    r.ws2 = (float *)dup(s.ws2);
    r.cperm = (uint32_t *)dup(s.cperm);
    r.bperm = dup(s.bperm);
    r.pad_out = dup(s.pad_out);
    for (size_t i = 0; i < s.pp.size(); i++) r.pp[i] = dup(s.pp[i]);
    if (!s.pp.empty()) {  // the whole-matrix stand-ins point at part 0 (upload_col_parts)
        r.col = r.pp[MP_PART_COL];
        r.val = r.pp[MP_PART_VAL];
    }
    p.dev.replicas.push_back(r);
}

void memset_rows(void *C, uint64_t lo, uint64_t hi, uint32_t N, size_t e, hipStream_t stream) {
    HIP_OK(hipMemsetAsync((char *)C + lo * N * e, 0, (hi - lo) * N * e, stream));
}

void combine_parts(const void *const *parts, const uint32_t *rows, uint32_t n, void *C, uint64_t row0, uint64_t P,
                   uint32_t N, int dtype, hipStream_t stream) {
    GS_CHECK(P * N < (1ull << 40) && n > 0, "combine_parts: bad sizes");
    const uint64_t total = P * N;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((total + 255) / 256, 4096);
    if (blocks == 0) return;
    if (dtype == 0)
        hipLaunchKernelGGL(gsk::k_combine_parts<float>, dim3(blocks), dim3(256), 0, stream,
                           (const float *const *)parts, rows, n, (float *)C + row0 * N, total, N);
    else
        hipLaunchKernelGGL(gsk::k_combine_parts<gsk::f16>, dim3(blocks), dim3(256), 0, stream,
                           (const gsk::f16 *const *)parts, rows, n, (gsk::f16 *)C + row0 * N, total, N);
    HIP_OK(hipGetLastError());
}

void free_device(plan_state &p) {
    if (!p.dev.allocations.empty()) (void)hipSetDevice(p.dev.device);
    for (void *x : p.dev.allocations) (void)hipFree(x);
    p.dev.allocations.clear();
    p.dev.replicas.clear();
    p.uploaded = false;
}

static void launch_body(plan_state &p, int replica, const void *B, void *C, uint32_t N, hipStream_t stream) {
    if (p.dev.nm) {
        launch_nm(p, p.dev.replicas[replica], B, C, N, stream);
        return;
    }
    if (p.dev.mfma && N == p.dev.lds_N) {
        launch_mfma(p, p.dev.replicas[replica], B, C, N, stream);
        return;
    }
    if (!p.dev.replicas[replica].col) {  // matrix-core plan at another dense width
        hipStreamCaptureStatus cs = hipStreamCaptureStatusNone;
        HIP_OK(hipStreamIsCapturing(stream, &cs));
        GS_CHECK(cs == hipStreamCaptureStatusNone,
                 "the first gs_spmm of a matrix-core plan at N != its tile width uploads its CSR "
                 "synchronously: run it once outside stream capture");
        ensure_csr(p);
    }
    launch_gather(p, p.dev.replicas[replica], B, C, N, stream);
}

void launch_spmm(plan_state &p, int replica, const void *B, void *C, uint32_t N, hipStream_t stream) {
    GS_CHECK(p.uploaded, "plan is not on the device");
    GS_CHECK(replica >= 0 && (size_t)replica < p.dev.replicas.size(), "bad replica index");
    GS_CHECK(N >= 1, "N >= 1");
    if (p.dev.pad_rows) {
        GS_CHECK(N <= p.dev.pad_N, "row-padded plan built for N=" + std::to_string(p.dev.pad_N) +
                                       ": its scratch output holds no wider B (re-run the pipeline for this N)");
        void *scr = p.dev.replicas[replica].pad_out;
        launch_body(p, replica, B, scr, N, stream);
        HIP_OK(hipGetLastError());
        HIP_OK(hipMemcpyAsync(C, scr, (size_t)p.M * N * (p.dev.dtype == 0 ? 4u : 2u), hipMemcpyDeviceToDevice, stream));
        return;
    }
    launch_body(p, replica, B, C, N, stream);
}

}  // namespace gs
