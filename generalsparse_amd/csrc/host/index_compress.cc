// index_compress.cc -- see index_compress.hpp (code_generator.cc:2618-3063).
#include "index_compress.hpp"

#include <algorithm>

namespace gs {

namespace {

// :2618-2640 (n >= 2; the reference reads a[1] unconditionally)
bool if_linear(const std::vector<uint64_t> &a) {
    const uint64_t coef = a[1] - a[0];
    for (size_t i = 0; i + 1 < a.size(); i++)
        if (a[i + 1] - a[i] != coef) return false;
    return true;
}

// :2642-2670: the run count is checked when a run starts
bool if_branch(const std::vector<uint64_t> &a, int64_t branch_max) {
    uint64_t item = a[0], count = 1;
    for (uint64_t x : a)
        if (x != item) {
            count += 1;
            item = x;
            if ((int64_t)count >= branch_max) return false;
        }
    return true;
}

// :2672-2715: the cycle is the LAST index i >= 1 holding a[0]
bool if_cycle_linear(const std::vector<uint64_t> &a) {
    const uint64_t coef = a[1] - a[0], icpt = a[0];
    uint64_t cycle = 1;
    for (size_t i = 1; i < a.size(); i++)
        if (a[i] == icpt) cycle = i;
    for (size_t i = 0; i < a.size(); i++) {
        const uint64_t in = i % cycle;
        if (in == 0 && a[i] != icpt) return false;
        if (in != 0 && (a[i] - icpt) / in != coef) return false;
    }
    return true;
}

// :2717-2760: the cycle is the first index whose value differs from a[0] (which must not
// decrease); accepted when every later value differs from a[0] by a multiple of its cycle id
bool if_cycle_increase(const std::vector<uint64_t> &a) {
    const uint64_t item1 = a[0];
    uint64_t cycle = 1;
    for (size_t i = 1; i < a.size(); i++)
        if (a[i] != item1) {
            if (a[i] < item1) return false;
            cycle = i;
            break;
        }
    if (a.size() % cycle != 0) return false;
    for (size_t i = 0; i < a.size(); i++) {
        const uint64_t id = i / cycle;
        if (id != 0 && (a[i] - item1) % id != 0) return false;
    }
    return true;
}

// :2762-2824: least squares in double, truncated to long; residuals shifted to >= 0
bool if_residual(const std::vector<uint64_t> &a, data_type type_ori, index_compression &c) {
    double t1 = 0, t2 = 0, t3 = 0, t4 = 0;
    const double n = (double)a.size();
    for (uint64_t i = 0; i < a.size(); i++) {
        const uint64_t item = a[i];
        t1 += (double)(i * i);
        t2 += (double)i;
        t3 += (double)(i * item);
        t4 += (double)item;
    }
    const double den = t1 * n - t2 * t2;
    const double fa = (t3 * n - t2 * t4) / den, fb = (t1 * t4 - t2 * t3) / den;
    const int64_t aa = (int64_t)fa;
    int64_t bb = (int64_t)fb;
    uint64_t max1 = 0, max2 = 0;
    for (uint64_t i = 0; i < a.size(); i++) {
        const int64_t err = (int64_t)(a[i] - (uint64_t)aa * i - (uint64_t)bb);
        if (err >= 0) {
            if ((uint64_t)err > max1) max1 = (uint64_t)err;
        } else if ((uint64_t)(-err) > max2) {
            max2 = (uint64_t)(-err);
        }
    }
    bb -= (int64_t)max2;
    if (find_most_suitable_data_type(max1 + max2) >= type_ori) return false;
    c.aa = aa;
    c.bb = bb;
    c.res.resize(a.size());
    for (uint64_t i = 0; i < a.size(); i++) c.res[i] = a[i] - (uint64_t)aa * i - (uint64_t)bb;
    return true;
}

}  // namespace

index_compression analyze_index_compression(const std::vector<uint64_t> &a, data_type type_ori, int64_t branch_max) {
    index_compression c;
    if (a.size() < 2) return c;  // the reference reads a[1] (and divides by zero in the fit)
    if (if_linear(a)) {
        c.kind = "linear";  // get_linear_compress :2826-2853
        c.coef = a[1] - a[0];
        c.intercept = a[0];
    } else if (if_branch(a, branch_max)) {
        c.kind = "branch";  // get_branch_compress :2855-2912
        c.lo.push_back(0);
        c.val.push_back(a[0]);
        for (uint64_t i = 0; i < a.size(); i++)
            if (a[i] != c.val.back()) {
                c.hi.push_back(i - 1);
                c.lo.push_back(i);
                c.val.push_back(a[i]);
            }
        c.hi.push_back(a.size() - 1);
    } else if (if_cycle_linear(a)) {
        c.kind = "cycle_linear";  // get_cycle_linear_compress :2914-2958 (cycle: last i >= 0 with a[0])
        c.coef = a[1] - a[0];
        c.intercept = a[0];
        for (uint64_t i = 0; i < a.size(); i++)
            if (a[i] == c.intercept) c.cycle = i;
    } else if (if_cycle_increase(a)) {
        c.kind = "cycle_increase";  // get_cycle_increase_compress :2960-2989
        c.intercept = a[0];
        for (uint64_t i = 0; i < a.size(); i++)
            if (a[i] != a[0]) {
                c.cycle = i;
                c.coef = a[i] - a[0];
                break;
            }
    } else if (if_residual(a, type_ori, c)) {
        c.kind = "residual";
    }
    if (c.kind != "none") {
        c.exact = (c.kind != "cycle_linear" || c.cycle != 0) && (c.kind != "cycle_increase" || c.cycle != 0);
        for (uint64_t i = 0; c.exact && i < a.size(); i++) c.exact = decode_index_compression(c, i) == a[i];
    }
    return c;
}

index_compression analyze_index_compression(meta_data_set &m, POS_TYPE pos, const std::string &name, int sub) {
    auto arr = m.get_element(pos, name, sub)->meta_data_arr;
    const config_t cfg = get_config();
    if (!cfg.MODEL_DRIVEN_COMPRESS || arr->get_data_type() == FLOAT || arr->get_data_type() == DOUBLE)
        return index_compression();
    index_compression c = analyze_index_compression(m.u(pos, name, sub), arr->get_compress_data_type(),
                                                    cfg.BRANCH_COMPRESS_MAX_SIZE);
    if (c.kind == "residual" && !m.is_exist(pos, name + "_res", sub))
        m.add_element(pos, name + "_res", sub, std::make_shared<universal_array>(c.res));
    return c;
}

uint64_t decode_index_compression(const index_compression &c, uint64_t i) {
    if (c.kind == "linear") return c.coef * i + c.intercept;
    if (c.kind == "branch") {
        for (size_t b = 0; b < c.lo.size(); b++)
            if (i >= c.lo[b] && i <= c.hi[b]) return c.val[b];
        return 0;
    }
    if (c.kind == "cycle_linear") return c.cycle ? (i % c.cycle) * c.coef + c.intercept : 0;
    if (c.kind == "cycle_increase") return c.cycle ? (i / c.cycle) * c.coef + c.intercept : 0;
    if (c.kind == "residual") return (uint64_t)c.aa * i + (uint64_t)c.bb + (i < c.res.size() ? c.res[i] : 0);
    return 0;
}

std::string code_of_index_compression(const index_compression &c, const std::string &idx, const std::string &res_name) {
    auto u = [](uint64_t x) { return std::to_string(x); };
    if (c.kind == "linear") {  // :2836-2851
        std::string r = c.coef == 0 ? u(c.intercept) : (c.coef != 1 ? u(c.coef) + " * (" + idx + ")" : idx);
        if (c.coef != 0 && c.intercept != 0) r += " + " + u(c.intercept);
        return r;
    }
    if (c.kind == "branch") {  // if-chain of index ranges
        std::string r;
        for (size_t b = 0; b < c.lo.size(); b++) {
            const std::string cond = c.lo[b] == c.hi[b] ? idx + " == " + u(c.lo[b])
                                                        : idx + " >= " + u(c.lo[b]) + " && " + idx + " <= " + u(c.hi[b]);
            r += "(" + cond + ") ? " + u(c.val[b]) + " : ";
        }
        return r + "0";
    }
    if (c.kind == "cycle_linear" || c.kind == "cycle_increase") {  // :2946-2952, :2979-2985
        std::string r = "( (" + idx + ") " + (c.kind == "cycle_linear" ? "% " : "/ ") + u(c.cycle) + " ) * " + u(c.coef);
        if (c.intercept != 0) r += " + " + u(c.intercept);
        return r;
    }
    if (c.kind == "residual")  // :3045-3060
        return std::to_string(c.aa) + " * (" + idx + ") + (" + std::to_string(c.bb) + ") + " + res_name + "[" + idx + "]";
    return "";
}

bool device_formula_of(const index_compression &c, gsk::idx_formula &f) {
    f = gsk::idx_formula();
    if (!c.exact) return false;
    auto fits = [](uint64_t x) { return x <= 0xffffffffull; };
    if (c.kind == "linear" || c.kind == "cycle_linear" || c.kind == "cycle_increase") {
        if (!fits(c.coef) || !fits(c.intercept) || !fits(c.cycle)) return false;
        f.kind = c.kind == "linear" ? gsk::IDX_LINEAR : (c.kind == "cycle_linear" ? gsk::IDX_CYCLE_LINEAR : gsk::IDX_CYCLE_INCREASE);
        f.coef = (uint32_t)c.coef;
        f.intercept = (uint32_t)c.intercept;
        f.cycle = c.kind == "linear" ? 1u : (uint32_t)c.cycle;
        return true;
    }
    if (c.kind == "branch") {
        if (c.lo.size() > (size_t)gsk::kIdxBranchMax) return false;
        for (size_t b = 0; b < c.lo.size(); b++)
            if (!fits(c.lo[b]) || !fits(c.val[b])) return false;
        f.kind = gsk::IDX_BRANCH;
        f.n_runs = (uint32_t)c.lo.size();
        for (size_t b = 0; b < c.lo.size(); b++) {
            f.lo[b] = (uint32_t)c.lo[b];
            f.val[b] = (uint32_t)c.val[b];
        }
        return true;
    }
    if (c.kind == "residual") {
        uint64_t mx = 0;
        for (uint64_t r : c.res) mx = std::max(mx, r);
        if (mx > 0xffff) return false;
        f.kind = mx <= 0xff ? gsk::IDX_RESIDUAL_U8 : gsk::IDX_RESIDUAL_U16;
        f.coef = (uint32_t)(uint64_t)c.aa;  // mod 2^32: the decoded values are < 2^32
        f.intercept = (uint32_t)(uint64_t)c.bb;
        return true;
    }
    return false;
}

std::string code_of_device_formula(const gsk::idx_formula &f) {
    auto u = [](uint32_t x) { return std::to_string(x) + "u"; };
    std::string r = "gsk::idx_formula{" + u(f.kind) + ", " + u(f.coef) + ", " + u(f.intercept) + ", " + u(f.cycle) + ", " +
                    u(f.n_runs) + ", {";
    for (int b = 0; b < gsk::kIdxBranchMax; b++) r += (b ? ", " : "") + u(f.lo[b]);
    r += "}, {";
    for (int b = 0; b < gsk::kIdxBranchMax; b++) r += (b ? ", " : "") + u(f.val[b]);
    return r + "}}";
}

}  // namespace gs
