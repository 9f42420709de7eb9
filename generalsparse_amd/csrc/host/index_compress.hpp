// index_compress.hpp -- model-driven index compression of plan arrays (SURVEY §8f
// rank 1; code_generator.cc:2618-3063 of the reference, arr_optimization.cc).
//
// The reference decides, per integer metadata array a kernel reads, whether the array
// can be replaced by an expression of the index (tried in this order,
// code_generator.cc:16-40 / 3067-3085):
//   linear          a[i] = coef * i + a[0]                       (:2618-2640)
//   branch          fewer than BRANCH_COMPRESS_MAX_SIZE runs      (:2642-2670)
//   cycle_linear    a[i] = (i % cycle) * coef + a[0]              (:2672-2715)
//   cycle_increase  a[i] = (i / cycle) * k + a[0]                 (:2717-2760)
//   residual        a[i] = aa * i + bb + res[i], res narrower     (:2762-2824)
// with the reference's unsigned 64-bit arithmetic.  Its acceptance tests for
// cycle_increase (divisibility only) and cycle_linear (integer division) admit arrays
// the emitted formula does not reproduce; `exact` records whether the formula
// reproduces the array, and the build's emitted programs only use exact formulas.
#pragma once

#include "gs_core.hpp"
#include "../hip_code/idx_formula.hpp"

namespace gs {

struct index_compression {
    std::string kind = "none";  // none | linear | branch | cycle_linear | cycle_increase | residual
    uint64_t coef = 0, intercept = 0, cycle = 0;
    std::vector<uint64_t> lo, hi, val;  // branch runs [lo, hi] -> val
    int64_t aa = 0, bb = 0;             // residual: aa * i + bb + res[i]
    std::vector<uint64_t> res;
    bool exact = false;                 // the formula reproduces every element
};

// decision + parameters for one array (type_ori: the array's compressed data type)
index_compression analyze_index_compression(const std::vector<uint64_t> &a, data_type type_ori, int64_t branch_max);
// for a plan array: honours MODEL_DRIVEN_COMPRESS (off -> "none"); a residual adds
// "<name>_res" to the metadata set (code_generator.cc:2808-2822)
index_compression analyze_index_compression(meta_data_set &m, POS_TYPE pos, const std::string &name, int sub);
uint64_t decode_index_compression(const index_compression &c, uint64_t i);
// the expression the generated kernel evaluates (get_*_compress, :2826-3063)
std::string code_of_index_compression(const index_compression &c, const std::string &idx, const std::string &res_name);
// the kernel-argument form of an exact compression (hip_code/idx_formula.hpp): false when
// the device kernels cannot evaluate it (not exact, values or constants beyond 32 bits,
// more than kIdxBranchMax runs, residuals wider than u16)
bool device_formula_of(const index_compression &c, gsk::idx_formula &f);
// its C++ initializer, for emitted programs
std::string code_of_device_formula(const gsk::idx_formula &f);

}  // namespace gs
