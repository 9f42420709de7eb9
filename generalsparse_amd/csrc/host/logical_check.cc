// logical_check -- cross-array consistency of a plan's metadata set
// (metadata_set.cc:806-1890; token_test asserts it after every pipeline,
// token_test.cc:517-1541).
//
// The reference's checks are restated (array lengths, begin <= end, the first and last
// entries of first_nz/first_row agreeing across levels, first_BMT/first_BMW pointing at
// the child whose start equals the parent's, first_nz_indices_without_ending == the
// THREAD starts, the BMT_size_of_each_blk walk).  Its relative-vs-absolute checks only
// count mismatches (metadata_set.cc:1302-1479: "k+1 == parents-1"); here every child
// start is checked exactly: child_abs[j] == child_rel[j] + parent_abs[parent of j], the
// parent of j taken from the parent's first_BMT/first_BMW indices, or from the nz range
// that holds the child's start.  Also checked (the build's): nz_row_indices
// non-decreasing, columns inside the matrix, every first_nz array non-decreasing from 0
// to the stored nnz.  Returns "" when the plan is consistent, else the first violation.
#include "operator.hpp"

#include <algorithm>
#include <cctype>
#include <cstdlib>
#include <sstream>

namespace gs {

namespace {

struct level_arrays {
    const std::vector<uint64_t> *nz = nullptr, *row = nullptr, *row_we = nullptr, *bmt = nullptr, *bmw = nullptr,
                                *bsize = nullptr, *nz_rel_bmtb = nullptr, *row_rel_bmtb = nullptr,
                                *nz_rel_bmw = nullptr, *row_rel_bmw = nullptr;
};

const std::vector<uint64_t> *arr(const meta_data_set &m, POS_TYPE p, const char *name, int sub) {
    if (!m.is_exist(p, name, sub)) return nullptr;
    auto e = m.get_element(p, name, sub)->meta_data_arr;
    return e->is_float() ? nullptr : &e->u();
}

std::string where(const char *what, int sub) {
    std::ostringstream o;
    o << what << " (sub-matrix " << sub << ")";
    return o.str();
}

// parent index of every child start: from the parent's first-child indices when present
// (pc[p] = first child of parent p), else by the nz range holding the child's start
std::vector<uint64_t> parents_of(const std::vector<uint64_t> &child_nz, const std::vector<uint64_t> &parent_nz,
                                 const std::vector<uint64_t> *pc, uint64_t n_children) {
    std::vector<uint64_t> par(n_children, 0);
    if (pc && pc->size() >= 2) {
        for (uint64_t p = 0; p + 1 < pc->size(); p++)
            for (uint64_t j = (*pc)[p]; j < (*pc)[p + 1] && j < n_children; j++) par[j] = p;
        return par;
    }
    uint64_t p = 0;
    for (uint64_t j = 0; j < n_children; j++) {
        while (p + 2 < parent_nz.size() && child_nz[j] >= parent_nz[p + 1]) p++;
        par[j] = p;
    }
    return par;
}

}  // namespace

std::string logical_check(const meta_data_set &m) {
    // sub-matrix ids present in the set
    std::vector<int> subs;
    for (const auto &k : m.keys()) {
        const auto us = k.find_last_of('_');
        if (us == std::string::npos) continue;
        const std::string tail = k.substr(us + 1);
        if (tail.empty() || (tail[0] != '-' && !isdigit((unsigned char)tail[0]))) continue;
        const int s = std::atoi(tail.c_str());
        if (s >= 0 && std::find(subs.begin(), subs.end(), s) == subs.end()) subs.push_back(s);
    }
    for (int i : subs) {
        const auto *row = arr(m, GLOBAL_META, "nz_row_indices", i), *col = arr(m, GLOBAL_META, "nz_col_indices", i);
        if (!row || !col) continue;  // a divided-away sub-matrix keeps only its boundaries
        if (row->size() != col->size()) return where("nz_col_indices length invalid", i);
        if (m.is_exist(GLOBAL_META, "nz_vals", i) &&
            m.get_element(GLOBAL_META, "nz_vals", i)->meta_data_arr->get_len() != row->size())
            return where("nz_vals length invalid", i);
        const uint64_t nnz = row->size();
        for (uint64_t e = 1; e < nnz; e++)
            if ((*row)[e] < (*row)[e - 1]) return where("nz_row_indices not sorted", i);
        if (m.is_exist(GLOBAL_META, "begin_row_index", i) && m.is_exist(GLOBAL_META, "end_row_index", i) &&
            m.scalar(GLOBAL_META, "begin_row_index", i) > m.scalar(GLOBAL_META, "end_row_index", i))
            return where("begin_row_index and end_row_index invalid", i);
        if (m.is_exist(GLOBAL_META, "begin_col_index", i) && m.is_exist(GLOBAL_META, "end_col_index", i)) {
            const uint64_t b = m.scalar(GLOBAL_META, "begin_col_index", i), e = m.scalar(GLOBAL_META, "end_col_index", i);
            if (b > e) return where("begin_col_index and end_col_index invalid", i);
            for (uint64_t c : *col)
                if (c > e - b) return where("nz_col_indices outside the sub-matrix's columns", i);
        }

        level_arrays L[3];  // TBLOCK, WARP, THREAD
        const POS_TYPE pos[3] = {TBLOCK_META, WARP_META, THREAD_META};
        for (int l = 0; l < 3; l++) {
            L[l].nz = arr(m, pos[l], "first_nz_indices", i);
            L[l].row = arr(m, pos[l], "first_row_indices", i);
            L[l].row_we = arr(m, pos[l], "first_row_indices_without_ending", i);
            L[l].bmt = arr(m, pos[l], "first_BMT_indices", i);
            L[l].bmw = arr(m, pos[l], "first_BMW_indices", i);
            L[l].bsize = arr(m, pos[l], "BMT_size_of_each_blk", i);
            L[l].nz_rel_bmtb = arr(m, pos[l], "first_nz_indices_relative_to_BMTB", i);
            L[l].row_rel_bmtb = arr(m, pos[l], "first_row_indices_relative_to_BMTB", i);
            L[l].nz_rel_bmw = arr(m, pos[l], "first_nz_indices_relative_to_BMW", i);
            L[l].row_rel_bmw = arr(m, pos[l], "first_row_indices_relative_to_BMW", i);
        }
        const char *lname[3] = {"TBLOCK", "WARP", "THREAD"};
        // BMWs / BMTBs merged from col-direction BMTs (first_row_indices_without_ending):
        // get_begin_rows_after_merge_thread.cc:39-44 walks j < len - 1 over the ending-less
        // rows and first_nz_indices over j < len, so when n_BMT - 1 is a multiple of the
        // merge size the row array comes out one short -- the group starts without an
        // ending.  The reference's tests check the plan before that operator only
        // (token_test.cc:1278); here the short array is checked as what it is.
        for (int l = 0; l < 2; l++)
            if (L[l].row && L[l].nz && L[l].bmt && L[2].row_we && L[l].row->size() + 1 == L[l].nz->size() &&
                !L[l].row_we) {
                L[l].row_we = L[l].row;
                L[l].row = nullptr;
            }
        for (int l = 0; l < 3; l++) {
            const auto *nz = L[l].nz;
            if (!nz) continue;
            std::string lv = std::string(" in ") + lname[l];
            if (nz->empty() || (*nz)[0] != 0) return where(("first_nz_indices must start at 0" + lv).c_str(), i);
            for (size_t j = 1; j < nz->size(); j++)
                if ((*nz)[j] < (*nz)[j - 1]) return where(("first_nz_indices decreasing" + lv).c_str(), i);
            if (nz->back() != nnz) return where(("first_nz_indices must end at the stored nnz" + lv).c_str(), i);
            if (L[l].row && L[l].row->size() != nz->size())
                return where(("first_row_indices or first_nz_indices invalid" + lv).c_str(), i);
            if (L[l].row_we && L[l].row_we->size() + 1 != nz->size())
                return where(("first_row_indices_without_ending or first_nz_indices invalid" + lv).c_str(), i);
            if (L[l].row)
                for (size_t j = 1; j < L[l].row->size(); j++)
                    if ((*L[l].row)[j] < (*L[l].row)[j - 1])
                        return where(("first_row_indices decreasing" + lv).c_str(), i);
            if (L[l].bsize && L[l].bsize->size() + 1 != nz->size())
                return where(("first_nz_indices or BMT_size_of_each_blk invalid" + lv).c_str(), i);
            if (L[l].bmt && L[l].bmt->size() != nz->size())
                return where(("first_BMT_indices or first_nz_indices invalid" + lv).c_str(), i);
        }
        // the units' entries lie in the units' rows (the build's check: a first_nz start that
        // lands in another row breaks it); col-direction BMTs inside a parent hold one row each
        // (row-direction units own rows [first_row[j], first_row[j+1]); the nnz-direction BMTs of
        // a bitmap plan share their boundary rows)
        const bool nnz_dir_thread = m.is_exist(THREAD_META, "thread_bit_map", i);
        for (int l = 0; l < 3; l++) {
            const auto *nz = L[l].nz;
            if (!nz) continue;
            // the BMWs of bitmap and col-direction plans group BMTs that split rows; units of a
            // fixed number of nonzeros (nnz-direction blocking at this level or below) split
            // rows too
            bool fixed_nnz = nz->size() >= 3;
            for (size_t j = 0; fixed_nnz && j + 2 < nz->size(); j++)
                fixed_nnz = (*nz)[j + 1] - (*nz)[j] == (*nz)[1] - (*nz)[0];
            for (int d = l + 1; d < 3 && !fixed_nnz; d++) {
                const auto *dn = L[d].nz;
                bool f = dn && dn->size() >= 3;
                for (size_t j = 0; f && j + 2 < dn->size(); j++) f = (*dn)[j + 1] - (*dn)[j] == (*dn)[1] - (*dn)[0];
                fixed_nnz = f;
            }
            const bool shared_rows = nnz_dir_thread || L[2].row_we != nullptr || fixed_nnz;
            if (L[l].row)
                for (size_t j = 0; j + 1 < nz->size(); j++) {
                    if ((*nz)[j + 1] == (*nz)[j]) continue;
                    const uint64_t first = (*row)[(*nz)[j]], last = (*row)[(*nz)[j + 1] - 1];
                    const uint64_t lo = (*L[l].row)[j], hi = (*L[l].row)[j + 1];
                    // (the merge-thread operators end the last unit at the last row, not one past it)
                    if (first < lo || last > hi || (!shared_rows && last == hi && hi > lo && j + 2 < nz->size()))
                        return where((std::string("first_nz_indices and first_row_indices disagree with the rows in ") +
                                      lname[l]).c_str(), i);
                }
            if (L[l].row_we) {
                for (size_t j = 1; j < L[l].row_we->size(); j++)
                    if ((*L[l].row_we)[j] < (*L[l].row_we)[j - 1])
                        return where((std::string("first_row_indices_without_ending decreasing in ") + lname[l]).c_str(), i);
                if (l == 2 && (L[0].bmt || L[1].bmt))
                    for (size_t j = 0; j + 1 < nz->size(); j++)
                        for (uint64_t e = (*nz)[j]; e < (*nz)[j + 1]; e++)
                            if ((*row)[e] != (*L[l].row_we)[j])
                                return where("first_row_indices_without_ending disagrees with the rows of its BMT in THREAD", i);
            }
        }
        // first and last starts agree across levels (metadata_set.cc:1074-1119)
        for (int a = 0; a < 3; a++)
            for (int b = a + 1; b < 3; b++) {
                if (L[a].nz && L[b].nz && (L[a].nz->front() != L[b].nz->front() || L[a].nz->back() != L[b].nz->back()))
                    return where((std::string("first_nz_indices invalid in ") + lname[a] + " and " + lname[b]).c_str(), i);
                if (L[a].row && L[b].row && (L[a].row->front() != L[b].row->front() || L[a].row->back() != L[b].row->back()))
                    return where((std::string("first_row_indices invalid in ") + lname[a] + " and " + lname[b]).c_str(), i);
            }
        // first_nz_indices_without_ending (THREAD): the THREAD starts (metadata_set.cc:1689-1705)
        if (const auto *we = arr(m, THREAD_META, "first_nz_indices_without_ending", i)) {
            if (!L[2].nz || we->size() + 1 != L[2].nz->size())
                return where("first_nz_indices_without_ending or first_nz_indices invalid in THREAD", i);
            for (size_t j = 0; j < we->size(); j++)
                if ((*we)[j] != (*L[2].nz)[j]) return where("first_nz_indices_without_ending invalid in THREAD", i);
        }
        // parent -> first child: the child starting where the parent starts (metadata_set.cc:1651-1688, 1829-1889)
        for (int p = 0; p < 2; p++) {
            if (L[p].bmt && L[p].nz && L[2].nz)
                for (size_t j = 0; j < L[p].bmt->size(); j++) {
                    const uint64_t k = (*L[p].bmt)[j];
                    if (k >= L[2].nz->size() || (*L[p].nz)[j] != (*L[2].nz)[k])
                        return where((std::string("first_BMT_indices or first_nz_indices invalid in ") + lname[p]).c_str(), i);
                }
        }
        if (L[0].bmw && L[0].nz && L[1].nz) {
            if (L[0].bmw->size() != L[0].nz->size()) return where("first_BMW_indices or first_nz_indices invalid in TBLOCK", i);
            for (size_t j = 0; j < L[0].bmw->size(); j++) {
                const uint64_t k = (*L[0].bmw)[j];
                if (k >= L[1].nz->size() || (*L[0].nz)[j] != (*L[1].nz)[k])
                    return where("first_BMW_indices invalid in TBLOCK", i);
                if (L[0].row && L[1].row && (*L[0].row)[j] != (*L[1].row)[k])
                    return where("first_BMW_indices or first_row_indices invalid in TBLOCK and WARP", i);
            }
        }
        // BMT_size_of_each_blk: every BMT of a parent has the parent's size (the walk of
        // metadata_set.cc:1706-1792, checked BMT by BMT)
        for (int p = 0; p < 2; p++) {
            if (!L[p].bsize || !L[p].nz || !L[2].nz) continue;
            const auto par = parents_of(*L[2].nz, *L[p].nz, L[p].bmt, L[2].nz->size() - 1);
            for (size_t j = 0; j + 1 < L[2].nz->size(); j++) {
                const uint64_t sz = (*L[2].nz)[j + 1] - (*L[2].nz)[j], want = (*L[p].bsize)[par[j]];
                if (sz != want && !(sz < want && (*L[2].nz)[j + 1] == (*L[p].nz)[par[j] + 1]))
                    return where((std::string("BMT_size_of_each_blk invalid in ") + lname[p]).c_str(), i);
            }
        }
        // relative <-> absolute starts, exactly (the build's form of metadata_set.cc:1302-1479)
        struct rel_case { int child, parent; const std::vector<uint64_t> *rel; bool nz; const std::vector<uint64_t> *pc; };
        const rel_case cases[] = {
            {1, 0, L[1].nz_rel_bmtb, true, L[0].bmw}, {1, 0, L[1].row_rel_bmtb, false, L[0].bmw},
            {2, 0, L[2].nz_rel_bmtb, true, L[0].bmt}, {2, 0, L[2].row_rel_bmtb, false, L[0].bmt},
            {2, 1, L[2].nz_rel_bmw, true, L[1].bmt},  {2, 1, L[2].row_rel_bmw, false, L[1].bmt}};
        for (const auto &c : cases) {
            if (!c.rel) continue;
            const auto *cnz = L[c.child].nz, *pnz = L[c.parent].nz;
            const auto *cabs = c.nz ? cnz : (L[c.child].row ? L[c.child].row : L[c.child].row_we);
            const auto *pabs = c.nz ? pnz : L[c.parent].row;
            if (!cnz || !pnz || !cabs || !pabs) continue;
            const uint64_t nchild = cnz->size() - 1;
            if (c.rel->size() != nchild && c.rel->size() != cnz->size())
                return where((std::string(c.nz ? "first_nz_indices" : "first_row_indices") + "_relative_to_" +
                              (c.parent == 0 ? "BMTB" : "BMW") + " length invalid in " + lname[c.child]).c_str(), i);
            const auto par = parents_of(*cnz, *pnz, c.pc, nchild);
            for (uint64_t j = 0; j < nchild && j < c.rel->size() && j < cabs->size(); j++)
                if ((*cabs)[j] != (*c.rel)[j] + (*pabs)[par[j]])
                    return where((std::string(c.nz ? "first_nz_indices" : "first_row_indices") + "_relative_to_" +
                                  (c.parent == 0 ? "BMTB" : "BMW") + " disagrees with the absolute starts in " +
                                  lname[c.child]).c_str(), i);
        }
    }
    return "";
}

}  // namespace gs
