// plan_io.cc -- binary plan files: one file per compiled plan
// instead of the reference's text data_source/<id>/ directory (metadata_set.cc:517-571
// writes one number per line with endl flushes and sleep(1) calls).  Layout, all little
// endian: "GSPLAN02", the number of kernels, per kernel its sub-matrix id and the kernel
// spec the code generator selected (one per sub-matrix of a row division, §8f rank 3),
// the pipeline and matrix names, then every metadata array as (pos, name, sub, is_float,
// data_type, len, payload u64/f64).  "GSPLAN03" adds, per kernel after its sub-matrix id,
// the parent-indexed row range of a row_nz_matrix_div_operator sub-matrix (base, rows; -1
// otherwise).  "GSPLAN02" and "GSPLAN01" files (one kernel, sub-matrix 0) still load.
#include "gs_plan.hpp"

#include <cstdio>
#include <cstring>

namespace gs {

namespace {

struct writer {
    FILE *f;
    void raw(const void *p, size_t n) { GS_CHECK(std::fwrite(p, 1, n, f) == n, "plan file: write failed"); }
    void u64(uint64_t x) { raw(&x, 8); }
    void i64(int64_t x) { raw(&x, 8); }
    void str(const std::string &s) { u64(s.size()); raw(s.data(), s.size()); }
};

struct reader {
    FILE *f;
    void raw(void *p, size_t n) { GS_CHECK(std::fread(p, 1, n, f) == n, "plan file: truncated"); }
    uint64_t u64() { uint64_t x; raw(&x, 8); return x; }
    int64_t i64() { int64_t x; raw(&x, 8); return x; }
    std::string str() {
        uint64_t n = u64();
        GS_CHECK(n < (1u << 20), "plan file: bad string");
        std::string s(n, '\0');
        raw(&s[0], n);
        return s;
    }
};

const char kMagic1[8] = {'G', 'S', 'P', 'L', 'A', 'N', '0', '1'};
const char kMagic2[8] = {'G', 'S', 'P', 'L', 'A', 'N', '0', '2'};
const char kMagic3[8] = {'G', 'S', 'P', 'L', 'A', 'N', '0', '3'};

void write_spec(writer &w, const kernel_spec &s) {
    w.i64(s.family); w.i64(s.coarsen_factor); w.i64(s.sparse_coarsen_factor); w.i64(s.vector_width);
    w.i64(s.warp_segment); w.i64(s.tblock_parent); w.i64(s.row_sorted); w.i64(s.bitmap_parent);
    w.i64(s.merge_level); w.i64(s.work_size); w.i64(s.group_level); w.i64(!s.interleaved ? 0 : (s.interleave_parent == GLOBAL_META ? 1 : 2 + (int64_t)s.interleave_parent));
    w.u64(s.ref_grid[0]); w.u64(s.ref_grid[1]); w.u64(s.ref_block[0]); w.u64(s.ref_block[1]);
    w.u64(s.arrays.size());
    for (auto &a : s.arrays) w.str(a);
}

kernel_spec read_spec(reader &r) {
    kernel_spec s;
    s.family = (int)r.i64(); s.coarsen_factor = (int)r.i64(); s.sparse_coarsen_factor = (int)r.i64();
    s.vector_width = (int)r.i64(); s.warp_segment = r.i64() != 0; s.tblock_parent = r.i64() != 0;
    s.row_sorted = r.i64() != 0; s.bitmap_parent = (POS_TYPE)r.i64(); s.merge_level = (POS_TYPE)r.i64();
    s.work_size = (int)r.i64(); s.group_level = (POS_TYPE)r.i64(); const int64_t il = r.i64();  // 0 none, 1 GLOBAL parent, 2 + pos a TBLOCK / WARP parent
    s.interleaved = il != 0;
    s.interleave_parent = il >= 2 ? (int)(il - 2) : (int)GLOBAL_META;
    s.ref_grid[0] = (unsigned)r.u64(); s.ref_grid[1] = (unsigned)r.u64();
    s.ref_block[0] = (unsigned)r.u64(); s.ref_block[1] = (unsigned)r.u64();
    const uint64_t na = r.u64();
    GS_CHECK(na < 4096, "plan file: bad array list");
    for (uint64_t i = 0; i < na; i++) s.arrays.push_back(r.str());
    return s;
}

}  // namespace

void save_plan(const std::vector<const plan_state *> &ks, const std::string &path) {
    GS_CHECK(!ks.empty(), "save: no kernel");
    for (auto *k : ks) GS_CHECK(k->cg && k->cg->is_compiled(), "save: compile the plan first");
    const plan_state &p = *ks.front();
    FILE *f = std::fopen(path.c_str(), "wb");
    GS_CHECK(f, "cannot write " + path);
    writer w{f};
    try {
        w.raw(kMagic3, 8);
        w.u64(ks.size());
        for (auto *k : ks) {
            w.i64(k->cg->get_sub_matrix_id());
            w.i64(k->parent_row_base);
            w.u64(k->parent_rows);
            write_spec(w, k->cg->get_kernel_spec());
        }
        w.str(p.pipeline);
        w.str(p.meta->matrix_name);
        const auto keys = p.meta->keys();
        w.u64(keys.size());
        for (auto &k : keys) {
            auto it = p.meta->get_element(k);
            auto &arr = *it->meta_data_arr;
            w.i64(it->meta_position); w.str(it->name); w.i64(it->sub_matrix_id);
            w.i64(arr.is_float()); w.i64(arr.get_data_type()); w.u64(arr.get_len());
            if (arr.is_float()) {
                std::vector<double> v(arr.get_len());
                for (uint64_t i = 0; i < v.size(); i++) v[i] = arr.read_float_from_arr(i);
                w.raw(v.data(), v.size() * 8);
            } else {
                w.raw(arr.u().data(), arr.get_len() * 8);
            }
        }
    } catch (...) {
        std::fclose(f);
        throw;
    }
    GS_CHECK(std::fclose(f) == 0, "plan file: close failed");
}

std::shared_ptr<meta_data_set> load_plan(const std::string &path, std::vector<loaded_kernel> &specs,
                                         std::string &pipeline) {
    FILE *f = std::fopen(path.c_str(), "rb");
    GS_CHECK(f, "cannot read " + path);
    reader r{f};
    std::shared_ptr<meta_data_set> m;
    try {
        char mg[8];
        r.raw(mg, 8);
        const bool v1 = std::memcmp(mg, kMagic1, 8) == 0, v3 = std::memcmp(mg, kMagic3, 8) == 0;
        GS_CHECK(v1 || v3 || std::memcmp(mg, kMagic2, 8) == 0, "not a generalsparse_amd plan file: " + path);
        specs.clear();
        const uint64_t nk = v1 ? 1 : r.u64();
        GS_CHECK(nk >= 1 && nk < 4096, "plan file: bad kernel count");
        for (uint64_t i = 0; i < nk; i++) {
            loaded_kernel k;
            k.sub = v1 ? 0 : (int)r.i64();
            if (v3) {
                k.parent_row_base = r.i64();
                k.parent_rows = r.u64();
            }
            k.spec = read_spec(r);
            specs.push_back(std::move(k));
        }
        pipeline = r.str();
        m = std::make_shared<meta_data_set>();
        m->matrix_name = r.str();
        const uint64_t na = r.u64();
        for (uint64_t i = 0; i < na; i++) {
            const POS_TYPE pos = (POS_TYPE)r.i64();
            const std::string name = r.str();
            const int sub = (int)r.i64();
            const bool is_f = r.i64() != 0;
            const data_type t = (data_type)r.i64();
            const uint64_t len = r.u64();
            GS_CHECK(len < (1ull << 40), "plan file: bad array length");
            if (is_f) {
                std::vector<double> v(len);
                r.raw(v.data(), len * 8);
                m->add_element(pos, name, sub, std::make_shared<universal_array>(std::move(v), t));
            } else {
                std::vector<uint64_t> v(len);
                r.raw(v.data(), len * 8);
                m->add_element(pos, name, sub, std::make_shared<universal_array>(std::move(v), t));
            }
        }
        for (auto &ks : specs)
            for (auto &a : ks.spec.arrays) GS_CHECK(m->is_exist(a), "plan file lacks kernel array " + a);
    } catch (...) {
        std::fclose(f);
        throw;
    }
    std::fclose(f);
    return m;
}

}  // namespace gs
