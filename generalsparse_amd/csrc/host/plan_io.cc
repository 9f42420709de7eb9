// plan_io.cc -- binary plan files: one file per compiled plan
// instead of the reference's text data_source/<id>/ directory (metadata_set.cc:517-571
// writes one number per line with endl flushes and sleep(1) calls).  Layout, all little
// endian: "GSPLAN01", the kernel spec the code generator selected, the plan's scalars,
// then every metadata array as (pos, name, sub, is_float, data_type, len, payload u64/f64).
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

const char kMagic[8] = {'G', 'S', 'P', 'L', 'A', 'N', '0', '1'};

}  // namespace

void save_plan(const plan_state &p, const std::string &path) {
    GS_CHECK(p.cg && p.cg->is_compiled(), "save: compile the plan first");
    FILE *f = std::fopen(path.c_str(), "wb");
    GS_CHECK(f, "cannot write " + path);
    writer w{f};
    try {
        w.raw(kMagic, 8);
        const kernel_spec &s = p.cg->get_kernel_spec();
        w.i64(s.family); w.i64(s.coarsen_factor); w.i64(s.sparse_coarsen_factor); w.i64(s.vector_width);
        w.i64(s.warp_segment); w.i64(s.tblock_parent); w.i64(s.row_sorted); w.i64(s.bitmap_parent);
        w.i64(s.merge_level); w.i64(s.work_size); w.i64(s.group_level); w.i64(s.interleaved);
        w.u64(s.ref_grid[0]); w.u64(s.ref_grid[1]); w.u64(s.ref_block[0]); w.u64(s.ref_block[1]);
        w.u64(s.arrays.size());
        for (auto &a : s.arrays) w.str(a);
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

void load_plan(plan_state &p, const std::string &path) {
    FILE *f = std::fopen(path.c_str(), "rb");
    GS_CHECK(f, "cannot read " + path);
    reader r{f};
    try {
        char mg[8];
        r.raw(mg, 8);
        GS_CHECK(std::memcmp(mg, kMagic, 8) == 0, "not a generalsparse_amd plan file: " + path);
        kernel_spec s;
        s.family = (int)r.i64(); s.coarsen_factor = (int)r.i64(); s.sparse_coarsen_factor = (int)r.i64();
        s.vector_width = (int)r.i64(); s.warp_segment = r.i64() != 0; s.tblock_parent = r.i64() != 0;
        s.row_sorted = r.i64() != 0; s.bitmap_parent = (POS_TYPE)r.i64(); s.merge_level = (POS_TYPE)r.i64();
        s.work_size = (int)r.i64(); s.group_level = (POS_TYPE)r.i64(); s.interleaved = r.i64() != 0;
        s.ref_grid[0] = (unsigned)r.u64(); s.ref_grid[1] = (unsigned)r.u64();
        s.ref_block[0] = (unsigned)r.u64(); s.ref_block[1] = (unsigned)r.u64();
        const uint64_t na = r.u64();
        GS_CHECK(na < 4096, "plan file: bad array list");
        for (uint64_t i = 0; i < na; i++) s.arrays.push_back(r.str());
        const std::string pipeline = r.str();
        auto m = std::make_shared<meta_data_set>();
        m->matrix_name = r.str();
        const uint64_t nk = r.u64();
        for (uint64_t i = 0; i < nk; i++) {
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
        for (auto &a : s.arrays) GS_CHECK(m->is_exist(a), "plan file lacks kernel array " + a);
        p.meta = m;
        p.cg = std::make_shared<code_generator>(m, 0);
        p.cg->restore_compiled(s);
        p.exec = std::make_shared<operator_executer>();
        p.pipeline = pipeline;
        p.M = m->scalar(GLOBAL_META, "origin_row_num", -1);
        p.K = m->scalar(GLOBAL_META, "origin_col_num", -1);
        p.nnz = m->scalar(GLOBAL_META, "origin_nnz_num", -1);
        p.uploaded = false;
    } catch (...) {
        std::fclose(f);
        throw;
    }
    std::fclose(f);
}

}  // namespace gs
