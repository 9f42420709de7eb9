// gs_core.cc -- see gs_core.hpp for the reference map.
#include "gs_core.hpp"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <sys/stat.h>

namespace gs {

std::string code_of_data_type(data_type t) {
    switch (t) {
        case CHAR: return "char";
        case UNSIGNED_CHAR: return "unsigned char";
        case SHORT: return "short";
        case UNSIGNED_SHORT: return "unsigned short";
        case INT: return "int";
        case UNSIGNED_INT: return "unsigned int";
        case LONG: return "long";
        case UNSIGNED_LONG: return "unsigned long";
        case LONG_LONG: return "long long";
        case UNSIGNED_LONG_LONG: return "unsigned long long";
        case HALF: return "__half";
        case HALF2: return "__half2";
        case FLOAT: return "float";
        case FLOAT2: return "float2";
        case FLOAT4: return "float4";
        case DOUBLE: return "double";
        case BOOL: return "bool";
        default: return "void";
    }
}

size_t size_of_data_type(data_type t) {
    switch (t) {
        case CHAR: case UNSIGNED_CHAR: case BOOL: return 1;
        case SHORT: case UNSIGNED_SHORT: case HALF: return 2;
        case INT: case UNSIGNED_INT: case FLOAT: case HALF2: return 4;
        case LONG: case UNSIGNED_LONG: case LONG_LONG: case UNSIGNED_LONG_LONG: case DOUBLE: return 8;
        default: return 8;
    }
}

data_type find_most_suitable_data_type(uint64_t m) {
    if (m <= 255) return UNSIGNED_CHAR;
    if (m <= 65535) return UNSIGNED_SHORT;
    if (m <= 4294967295ull) return UNSIGNED_INT;
    return UNSIGNED_LONG;
}

std::string convert_pos_type_to_string(POS_TYPE t) {
    switch (t) {
        case GLOBAL_META: return "GLOBAL_META";
        case TBLOCK_META: return "TBLOCK_META";
        case WARP_META: return "WARP_META";
        case THREAD_META: return "THREAD_META";
        case ROW_META: return "ROW_META";
        case COL_META: return "COL_META";
        case VAL_META: return "VAL_META";
        default: return "NONE_META";
    }
}

std::string get_metadata_item_name(POS_TYPE pos, const std::string &name, int sub) {
    return convert_pos_type_to_string(pos) + "_" + name + "_" + std::to_string(sub);
}

// ---------------------------------------------------------------- config
// switches that select kernels kept only in the experiments build (make -C csrc exp):
// measured slower than the default kernels, parity-tested there
bool experiments_key(const std::string &k) {
    return k == "MFMA_BM" || k == "NM_KS" || k == "MFMA_FLAGS" || k == "BM_V2" || k == "BM_KB" || k == "MP_ROWS" ||
           k == "KS_FORCE_TIMEOUT" || k == "KS_POS8" || k == "NM_V4" || k == "KS_PERSIST";
}

// a key / value the release build refuses, whether from set_config or a JSON config file
[[maybe_unused]] static bool refused_in_release(const std::string &k, int64_t value, bool is_true) {
    const bool on = value != 0 || is_true;
    return (on && experiments_key(k)) || (k == "KS_WAVES" && value != 8) || (k == "KS_APART" && value != 1 && !is_true);
}

namespace {
std::mutex g_cfg_mu;
bool g_cfg_loaded = false;
config_t g_cfg;

void apply_kv(config_t &c, const std::string &k, const std::string &v) {
    auto b = [&]() { return v == "true" || v == "1"; };
    auto i = [&]() { return (int64_t)std::atof(v.c_str()); };
    if (k == "DENSE_MATRIX_SIZE") c.DENSE_MATRIX_SIZE = i();
    else if (k == "VECTOR_WIDTH") c.VECTOR_WIDTH = i();
    else if (k == "HALF") c.HALF = b();
    else if (k == "PRECISE_OF_FLOAT") c.PRECISE_OF_FLOAT = v;
    else if (k == "ROOT_PATH_STR") c.ROOT_PATH_STR = v;
    else if (k == "DATA_SET") c.DATA_SET = v;
    else if (k == "OPERATOR_RUNTIME_CHECK") c.OPERATOR_RUNTIME_CHECK = b();
    else if (k == "PADDING_RATE_UP_BOUND") c.PADDING_RATE_UP_BOUND = i();
    else if (k == "DATA_TYPE_COMPRESS") c.DATA_TYPE_COMPRESS = b();
    else if (k == "BRANCH_COMPRESS_MAX_SIZE") c.BRANCH_COMPRESS_MAX_SIZE = i();
    else if (k == "FLOAT_RATE") c.FLOAT_RATE = i();
    else if (k == "GFLOPS_UP_BOUND") c.GFLOPS_UP_BOUND = std::atof(v.c_str());
    else if (k == "SHARED_MEM_TOTAL_SIZE") c.SHARED_MEM_TOTAL_SIZE = i();
    else if (k == "MAX_DIV_TIMES_OF_DIV") c.MAX_DIV_TIMES_OF_DIV = i();
    else if (k == "MFMA_GLDS") c.MFMA_GLDS = i();
    else if (k == "MFMA_GLDS_NBUF") c.MFMA_GLDS_NBUF = i();
    else if (k == "MFMA_COMPUTE_WAVES") c.MFMA_COMPUTE_WAVES = i();
    else if (k == "FORMAT_OF_MTX") c.FORMAT_OF_MTX = v;
    else if (k == "PERFORMANCE_FLAG") c.PERFORMANCE_FLAG = v;
    else if (k == "Graph_Algorithm") c.Graph_Algorithm = v;
    else if (k == "MODEL_DRIVEN_COMPRESS") c.MODEL_DRIVEN_COMPRESS = b();
    else if (k == "LDS_STAGE_B") c.LDS_STAGE_B = b();
    else if (k == "MFMA_TILES") c.MFMA_TILES = b();
    else if (k == "MFMA_MAX_FILL") c.MFMA_MAX_FILL = i();
    else if (k == "MFMA_KROT") c.MFMA_KROT = i();
    else if (k == "WARP_ROWS_GROUPS") c.WARP_ROWS_GROUPS = i();
    else if (k == "WARP_ROWS_CHUNKS") c.WARP_ROWS_CHUNKS = i();
    else if (k == "MFMA_KSPLIT") c.MFMA_KSPLIT = i();
    else if (k == "NM_MFMA") c.NM_MFMA = b();
    else if (k == "MFMA_KS") c.MFMA_KS = b();
    else if (k == "MFMA_BM") c.MFMA_BM = b();
    else if (k == "NM_KS") c.NM_KS = b();
    else if (k == "MFMA_FLAGS") c.MFMA_FLAGS = b();
    else if (k == "NM_SPLIT") c.NM_SPLIT = i();
    else if (k == "BM_SPLIT") c.BM_SPLIT = i();
    else if (k == "BM_WAVES") c.BM_WAVES = i();
    else if (k == "BM_V2") c.BM_V2 = b();
    else if (k == "BM_KB") c.BM_KB = b();
    else if (k == "KS_MIN_ROWS") c.KS_MIN_ROWS = i();
    else if (k == "KS_SPLIT") c.KS_SPLIT = i();
    else if (k == "KS_WAVES") c.KS_WAVES = i();
    else if (k == "KS_PRIO") c.KS_PRIO = i();
    else if (k == "KS_FORCE_TIMEOUT") c.KS_FORCE_TIMEOUT = i();
    else if (k == "KS_APART") c.KS_APART = i();
    else if (k == "NM_V4") c.NM_V4 = i();
    else if (k == "KS_POS8") c.KS_POS8 = i();
    else if (k == "KS_NT") c.KS_NT = i();
    else if (k == "NM_KROT") c.NM_KROT = i();
    else if (k == "NM_TILES") c.NM_TILES = i();
    else if (k == "LDS_KSPLIT") c.LDS_KSPLIT = i();
    else if (k == "LDS_DMA") c.LDS_DMA = i();
    else if (k == "MP_COL_PARTS") c.MP_COL_PARTS = i();
    else if (k == "MP_HUB_COLS") c.MP_HUB_COLS = i();
    else if (k == "KS_PERSIST") c.KS_PERSIST = i();
    else if (k == "KS_HEAD") c.KS_HEAD = i();
    else if (k == "NM_NT") c.NM_NT = i();
    else if (k == "MP_ROWS") c.MP_ROWS = b();
    else if (k == "MP_SOLO") c.MP_SOLO = i();
    else if (k == "MP_COL_PERM") c.MP_COL_PERM = i();
    else if (k == "MP_PERM_HOT") c.MP_PERM_HOT = i();
    else if (k == "MP_PERM_SCATTER") c.MP_PERM_SCATTER = i();
    // unknown keys are ignored, as the reference ignores 17 of its 36 keys
}

// minimal flat-JSON reader: {"KEY": value, ...} with string/number/bool values
void load_json(config_t &c, const std::string &path) {
    std::ifstream in(path);
    if (!in) return;
    std::stringstream ss;
    ss << in.rdbuf();
    std::string s = ss.str();
    size_t p = 0;
    while (true) {
        size_t q0 = s.find('"', p);
        if (q0 == std::string::npos) break;
        size_t q1 = s.find('"', q0 + 1);
        if (q1 == std::string::npos) break;
        std::string key = s.substr(q0 + 1, q1 - q0 - 1);
        size_t colon = s.find(':', q1);
        if (colon == std::string::npos) break;
        size_t v0 = s.find_first_not_of(" \t\r\n", colon + 1);
        if (v0 == std::string::npos) break;
        std::string val;
        if (s[v0] == '"') {
            size_t v1 = s.find('"', v0 + 1);
            val = s.substr(v0 + 1, v1 - v0 - 1);
            p = v1 + 1;
        } else {
            size_t v1 = s.find_first_of(",}\n", v0);
            val = s.substr(v0, v1 - v0);
            while (!val.empty() && isspace((unsigned char)val.back())) val.pop_back();
            p = v1;
        }
#ifndef GS_EXPERIMENTS
        // the experiments-build switches are refused here as in set_config: a plan built with
        // one would reach release kernels that do not read its layout
        if (refused_in_release(key, std::atoi(val.c_str()), val == "true"))
            throw gs_error(key + " in " + path + " selects an experiments-build kernel", -2);
#endif
        apply_kv(c, key, val);
    }
}

void ensure_loaded() {
    if (g_cfg_loaded) return;
    g_cfg = config_t();
    const char *env = std::getenv("GS_CONFIG");
    load_json(g_cfg, env ? env : "global_config.json");
    g_cfg_loaded = true;
}
}  // namespace

config_t get_config() {
    std::lock_guard<std::mutex> l(g_cfg_mu);
    ensure_loaded();
    return g_cfg;
}

void set_config(const std::string &key, int64_t value) {
#ifndef GS_EXPERIMENTS
    if (refused_in_release(key, value, false))
        throw gs_error(key + " selects an experiments-build kernel (make -C generalsparse_amd/csrc exp)", -2);
#endif
    std::lock_guard<std::mutex> l(g_cfg_mu);
    ensure_loaded();
    apply_kv(g_cfg, key, std::to_string(value));
}

int64_t get_config_int(const std::string &k) {
#ifdef GS_EXPERIMENTS
    if (k == "GS_EXPERIMENTS") return 1;
#else
    if (k == "GS_EXPERIMENTS") return 0;
#endif
    const config_t c = get_config();
#define GS_KEY(name) \
    if (k == #name) return (int64_t)c.name;
    GS_KEY(DENSE_MATRIX_SIZE) GS_KEY(VECTOR_WIDTH) GS_KEY(HALF) GS_KEY(OPERATOR_RUNTIME_CHECK)
    GS_KEY(PADDING_RATE_UP_BOUND) GS_KEY(DATA_TYPE_COMPRESS) GS_KEY(BRANCH_COMPRESS_MAX_SIZE) GS_KEY(FLOAT_RATE)
    GS_KEY(SHARED_MEM_TOTAL_SIZE) GS_KEY(MAX_DIV_TIMES_OF_DIV) GS_KEY(MFMA_GLDS) GS_KEY(MFMA_COMPUTE_WAVES)
    GS_KEY(MFMA_GLDS_NBUF) GS_KEY(MODEL_DRIVEN_COMPRESS) GS_KEY(LDS_STAGE_B) GS_KEY(MFMA_TILES) GS_KEY(MFMA_KROT)
    GS_KEY(WARP_ROWS_GROUPS) GS_KEY(WARP_ROWS_CHUNKS) GS_KEY(MFMA_MAX_FILL) GS_KEY(NM_MFMA) GS_KEY(MFMA_KSPLIT) GS_KEY(MFMA_KS)
    GS_KEY(NM_KS) GS_KEY(NM_SPLIT) GS_KEY(MFMA_FLAGS) GS_KEY(MFMA_BM) GS_KEY(BM_SPLIT) GS_KEY(BM_WAVES) GS_KEY(BM_V2) GS_KEY(BM_KB) GS_KEY(KS_MIN_ROWS) GS_KEY(KS_SPLIT) GS_KEY(KS_WAVES) GS_KEY(KS_PRIO) GS_KEY(KS_FORCE_TIMEOUT) GS_KEY(KS_APART) GS_KEY(NM_V4) GS_KEY(KS_POS8) GS_KEY(KS_NT) GS_KEY(NM_KROT) GS_KEY(NM_TILES) GS_KEY(LDS_KSPLIT) GS_KEY(LDS_DMA) GS_KEY(MP_COL_PARTS) GS_KEY(MP_HUB_COLS) GS_KEY(KS_PERSIST) GS_KEY(KS_HEAD) GS_KEY(NM_NT) GS_KEY(MP_ROWS) GS_KEY(MP_SOLO) GS_KEY(MP_COL_PERM) GS_KEY(MP_PERM_HOT) GS_KEY(MP_PERM_SCATTER)
#undef GS_KEY
    throw gs_error("get_config_int: no integer key " + k);
}

void set_config_str(const std::string &key, const std::string &value) {
    std::lock_guard<std::mutex> l(g_cfg_mu);
    ensure_loaded();
    apply_kv(g_cfg, key, value);
}

void reset_config() {
    std::lock_guard<std::mutex> l(g_cfg_mu);
    g_cfg_loaded = false;
}

// ---------------------------------------------------------------- arrays
universal_array::universal_array(std::vector<uint64_t> v, data_type t)
    : type_(t), is_float_(false), u_(std::move(v)) {}

universal_array::universal_array(std::vector<double> v, data_type t) : type_(t), is_float_(true), f_(std::move(v)) {
    GS_CHECK(t == FLOAT || t == DOUBLE, "float array type");
}

uint64_t universal_array::max_integer() const {
    uint64_t m = 0;
    for (uint64_t x : u_) m = std::max(m, x);
    return m;
}

data_type universal_array::get_compress_data_type() const {
    if (is_float_) return type_;
    if (!get_config().DATA_TYPE_COMPRESS) return type_;
    return find_most_suitable_data_type(max_integer());
}

void universal_array::output_2_file(const std::string &path) const {
    FILE *f = std::fopen(path.c_str(), "w");
    GS_CHECK(f, "cannot write " + path);
    std::vector<char> buf(1 << 20);
    std::setvbuf(f, buf.data(), _IOFBF, buf.size());
    if (is_float_) {
        for (double x : f_) {
            // struct.cc:2022-2025 clamps values <= 1e-10 to 0 (negatives included);
            // we keep the sign (documented deviation) and 6 significant digits.
            std::fprintf(f, "%.6g\n", std::fabs(x) <= 1e-10 ? 0.0 : x);
        }
    } else {
        for (uint64_t x : u_) std::fprintf(f, "%llu\n", (unsigned long long)x);
    }
    std::fclose(f);
}

// ---------------------------------------------------------------- set
void meta_data_set::add_element(POS_TYPE pos, const std::string &name, int sub, std::shared_ptr<universal_array> arr,
                                bool constant) {
    std::string key = get_metadata_item_name(pos, name, sub);
    GS_CHECK(data_map.count(key) == 0, "meta_data_set::add_element: key exists: " + key);
    auto it = std::make_shared<meta_data_item>();
    it->meta_data_arr = std::move(arr);
    it->meta_position = pos;
    it->name = name;
    it->sub_matrix_id = sub;
    it->is_constant = constant;
    data_map[key] = it;
}

void meta_data_set::add_scalar(POS_TYPE pos, const std::string &name, int sub, uint64_t v) {
    add_element(pos, name, sub, std::make_shared<universal_array>(std::vector<uint64_t>{v}), true);
}

void meta_data_set::remove_element(const std::string &key) {
    GS_CHECK(data_map.count(key) != 0, "meta_data_set::remove_element: no key " + key);
    data_map.erase(key);
}

void meta_data_set::remove_element(POS_TYPE pos, const std::string &name, int sub) {
    remove_element(get_metadata_item_name(pos, name, sub));
}

std::shared_ptr<meta_data_item> meta_data_set::get_element(const std::string &key) const {
    auto it = data_map.find(key);
    GS_CHECK(it != data_map.end(), "meta_data_set::get_element: no key " + key);
    return it->second;
}

std::shared_ptr<meta_data_item> meta_data_set::get_element(POS_TYPE pos, const std::string &name, int sub) const {
    return get_element(get_metadata_item_name(pos, name, sub));
}

bool meta_data_set::is_exist(POS_TYPE pos, const std::string &name, int sub) const {
    return is_exist(get_metadata_item_name(pos, name, sub));
}

int meta_data_set::count_of_metadata_of_diff_pos(POS_TYPE pos, int sub) const {
    int c = 0;
    for (auto &kv : data_map)
        if (kv.second->meta_position == pos && kv.second->sub_matrix_id == sub) c++;
    return c;
}

std::vector<std::string> meta_data_set::all_item_of_metadata_of_diff_pos(POS_TYPE pos, int sub) const {
    std::vector<std::string> r;
    for (auto &kv : data_map)
        if (kv.second->meta_position == pos && kv.second->sub_matrix_id == sub) r.push_back(kv.second->name);
    return r;
}

int meta_data_set::get_max_sub_matrix_id_of_data_item(POS_TYPE pos, const std::string &name) const {
    int mx = -1;
    for (auto &kv : data_map)
        if (kv.second->meta_position == pos && kv.second->name == name) mx = std::max(mx, kv.second->sub_matrix_id);
    return mx;
}

std::vector<std::string> meta_data_set::keys() const {
    std::vector<std::string> r;
    for (auto &kv : data_map) r.push_back(kv.first);
    return r;
}

uint64_t meta_data_set::output_format_to_dir(const std::string &root, const std::vector<std::string> &keys,
                                             std::string *dir_out) const {
    static std::atomic<uint64_t> counter{0};
    uint64_t id = (uint64_t)std::chrono::system_clock::now().time_since_epoch().count() % 1000000000ull * 100 +
                  (counter++ % 100) + 1;
    std::string base = root + "/data_source";
    ::mkdir(base.c_str(), 0755);
    std::string dir = base + "/" + std::to_string(id);
    GS_CHECK(::mkdir(dir.c_str(), 0755) == 0, "mkdir " + dir);
    for (auto &k : keys) get_element(k)->meta_data_arr->output_2_file(dir + "/" + k);
    if (dir_out) *dir_out = dir;
    return id;
}

// ---------------------------------------------------------------- reader
// Index bound of every entry point: the device layouts keep row / column COUNTS in 32 bits
// ((uint32_t)n_rows_aux, K < 2^32 in the MP_COL_PERM gate), so the largest index is 2^32 - 2
// and a dimension at most 2^32 - 1 (the reference's int reader keeps unsigned int,
// struct.cc:263-270).
static constexpr uint64_t kMaxIndex = 0xfffffffeull;

// one 1-based .mtx index token: decimal digits up to the next space / end of token, value >= 1
// (the reference's stoul would take "0" to an index of -1 and garbage to 0 - 1)
static uint64_t mtx_index(const char *tok, const char *end) {
    while (tok && tok < end && (*tok == ' ' || *tok == '\t')) tok++;
    GS_CHECK(tok && tok < end && *tok >= '0' && *tok <= '9', "malformed mtx index");
    char *stop = nullptr;
    uint64_t v = std::strtoull(tok, &stop, 10);
    GS_CHECK(stop == end || *stop == ' ' || *stop == '\t', "malformed mtx index");
    GS_CHECK(v >= 1 && v - 1 <= kMaxIndex, "mtx index out of range (1-based, at most 2^32 - 1)");
    return v - 1;
}

void get_matrix_index_and_val_from_file(const std::string &path, bool ones_values, coo_t &out) {
    std::unique_ptr<FILE, int (*)(FILE *)> fh(std::fopen(path.c_str(), "rb"), std::fclose);
    FILE *f = fh.get();
    GS_CHECK(f, "get_matrix_index_and_val_from_file: cannot open file " + path);
    out = coo_t();
    std::vector<char> buf(1 << 24);
    std::string carry;
    bool first = true;
    auto handle_line = [&](const char *s, size_t L) {
        // struct.cc:97: skip empty lines and lines starting with whitespace or '%'
        if (L == 0 || s[0] == ' ' || s[0] == '\t' || s[0] == '%' || s[0] == '\r') return;
        const char *tok[3] = {nullptr, nullptr, nullptr};
        int nt = 0;
        const char *p = s, *e = s + L;
        while (nt < 3 && p < e) {  // split on single spaces (struct.hpp:290)
            tok[nt++] = p;
            const char *sp = (const char *)std::memchr(p, ' ', e - p);
            if (!sp) break;
            p = sp + 1;
        }
        if (first) {  // struct.cc:104-110
            out.max_row_index = mtx_index(tok[0], e);
            out.max_col_index = nt > 1 ? mtx_index(tok[1], e) : 0;
            first = false;
            return;
        }
        GS_CHECK(nt >= 2, "malformed mtx line");
        uint64_t r = mtx_index(tok[0], e);
        uint64_t c = mtx_index(tok[1], e);
        float v = 1.0f;
        if (!ones_values && nt > 2) v = std::strtof(tok[2], nullptr);
        // struct.cc:120-131: entries must be row-sorted
        GS_CHECK(out.row.empty() || r >= out.row.back(), "mtx entries are not row-sorted (struct.cc:125)");
        out.row.push_back(r);
        out.col.push_back(c);
        out.val.push_back(v);
        if (r > out.max_row_index) out.max_row_index = r;
        if (c > out.max_col_index) out.max_col_index = c;
    };
    size_t n;
    while ((n = std::fread(buf.data(), 1, buf.size(), f)) > 0) {
        size_t start = 0;
        for (size_t i = 0; i < n; i++) {
            if (buf[i] == '\n') {
                if (!carry.empty()) {
                    carry.append(buf.data() + start, i - start);
                    size_t L = carry.size();
                    if (L && carry[L - 1] == '\r') L--;
                    handle_line(carry.data(), L);
                    carry.clear();
                } else {
                    size_t L = i - start;
                    if (L && buf[start + L - 1] == '\r') L--;
                    handle_line(buf.data() + start, L);
                }
                start = i + 1;
            }
        }
        carry.append(buf.data() + start, n - start);
    }
    if (!carry.empty()) handle_line(carry.data(), carry.size());
    GS_CHECK(!out.row.empty(), "empty matrix (struct.cc:258)");
}

static std::shared_ptr<meta_data_set> init_set(uint64_t max_row, uint64_t max_col, std::vector<uint64_t> row,
                                               std::vector<uint64_t> col, const std::vector<float> &val,
                                               const std::string &name) {
    GS_CHECK(!row.empty(), "empty matrix (struct.cc:258)");
    auto m = std::make_shared<meta_data_set>();
    m->matrix_name = name;
    uint64_t nnz = row.size();
    m->add_scalar(GLOBAL_META, "origin_row_num", -1, max_row + 1);
    m->add_scalar(GLOBAL_META, "origin_col_num", -1, max_col + 1);
    m->add_scalar(GLOBAL_META, "origin_nnz_num", -1, nnz);
    m->add_scalar(GLOBAL_META, "begin_row_index", 0, 0);
    m->add_scalar(GLOBAL_META, "begin_col_index", 0, 0);
    m->add_scalar(GLOBAL_META, "end_row_index", 0, max_row);
    m->add_scalar(GLOBAL_META, "end_col_index", 0, max_col);
    m->add_element(GLOBAL_META, "nz_row_indices", 0, std::make_shared<universal_array>(std::move(row)));
    m->add_element(GLOBAL_META, "nz_col_indices", 0, std::make_shared<universal_array>(std::move(col)));
    std::vector<double> v(val.begin(), val.end());
    m->add_element(GLOBAL_META, "nz_vals", 0, std::make_shared<universal_array>(std::move(v), FLOAT));
    return m;
}

std::shared_ptr<meta_data_set> create_init_metadata_set_from_file(const std::string &path, const std::string &name,
                                                                  bool ones_values) {
    coo_t c;
    get_matrix_index_and_val_from_file(path, ones_values, c);
    return init_set(c.max_row_index, c.max_col_index, std::move(c.row), std::move(c.col), c.val, name);
}

std::shared_ptr<meta_data_set> create_init_metadata_set_from_coo(uint64_t n_rows, uint64_t n_cols, uint64_t nnz,
                                                                 const uint64_t *row, const uint64_t *col,
                                                                 const float *val, const std::string &name) {
    GS_CHECK(nnz > 0, "empty matrix (struct.cc:258)");
    GS_CHECK(n_rows > 0 && n_cols > 0, "matrix dims must be positive");
    uint64_t max_row = n_rows - 1, max_col = n_cols - 1;
    std::vector<uint64_t> r(row, row + nnz), c(col, col + nnz);
    GS_CHECK(max_row <= kMaxIndex && max_col <= kMaxIndex, "matrix dims above 2^32 - 1");
    for (uint64_t i = 0; i < nnz; i++) {
        GS_CHECK(i == 0 || r[i] >= r[i - 1], "COO entries are not row-sorted (struct.cc:125)");
        GS_CHECK(r[i] <= kMaxIndex && c[i] <= kMaxIndex, "COO index out of range (at most 2^32 - 2)");
        max_row = std::max(max_row, r[i]);
        max_col = std::max(max_col, c[i]);
    }
    std::vector<float> v;
    if (val) v.assign(val, val + nnz);
    else v.assign(nnz, 1.0f);
    return init_set(max_row, max_col, std::move(r), std::move(c), v, name);
}

std::vector<uint64_t> get_nnz_of_each_row_in_spec_range(const std::vector<uint64_t> &rows, uint64_t begin_row,
                                                        uint64_t end_row, uint64_t begin_nz, uint64_t end_nz) {
    std::vector<uint64_t> cnt(end_row - begin_row + 1, 0);
    for (uint64_t i = begin_nz; i <= end_nz; i++) cnt[rows[i] - begin_row]++;
    return cnt;
}

uint64_t row_num_of_sub_matrix(const meta_data_set &m, int sub) {
    uint64_t b = m.scalar(GLOBAL_META, "begin_row_index", sub);
    uint64_t e = m.scalar(GLOBAL_META, "end_row_index", sub);
    const auto &r = m.u(GLOBAL_META, "nz_row_indices", sub);
    uint64_t real = b + r.back();
    if (e < real) e = real;
    GS_CHECK(e >= b, "end_row_index < begin_row_index");
    return e - b + 1;
}

}  // namespace gs
