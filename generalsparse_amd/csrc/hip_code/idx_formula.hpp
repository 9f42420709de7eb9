// hip_code/idx_formula.hpp -- an index array evaluated in the kernel instead of read
// (model-driven index compression).
//
// The reference's code generator replaces an integer metadata array by the expression
// its analysis found (code_generator.cc:2618-3063: get_linear_compress,
// get_branch_compress, get_cycle_linear_compress, get_cycle_increase_compress,
// get_residual_compress) and prints that expression into the generated kernel.  Here the
// kernels are compiled once, so the expression is data: a small by-value kernel argument
// naming the kind and its constants.  With kind != ARRAY the array is not uploaded at all
// (residual: only the narrow residual array is), which is the HBM traffic the reference's
// compression saves.  Arithmetic is mod 2^32: every device index array holds u32 values,
// so an exact formula evaluated mod 2^32 gives the same value.
#pragma once

#include <stdint.h>

namespace gsk {

enum idx_kind : uint32_t {
    IDX_ARRAY = 0,           // read a[i] (u32)
    IDX_LINEAR = 1,          // coef * i + intercept
    IDX_CYCLE_LINEAR = 2,    // (i % cycle) * coef + intercept
    IDX_CYCLE_INCREASE = 3,  // (i / cycle) * coef + intercept
    IDX_RESIDUAL_U8 = 4,     // coef * i + intercept + res8[i]   (a points at u8 residuals)
    IDX_RESIDUAL_U16 = 5,    // coef * i + intercept + res16[i]  (a points at u16 residuals)
    IDX_BRANCH = 6,          // val[b] for the last run b with lo[b] <= i (runs <= kIdxBranchMax)
};
constexpr int kIdxBranchMax = 4;

struct idx_formula {
    uint32_t kind = IDX_ARRAY;
    uint32_t coef = 0, intercept = 0, cycle = 1;
    uint32_t n_runs = 0;
    uint32_t lo[kIdxBranchMax] = {0, 0, 0, 0}, val[kIdxBranchMax] = {0, 0, 0, 0};
};

#if defined(__HIP__) || defined(__HIPCC__)
__device__ __forceinline__ uint32_t idx_eval(const uint32_t *__restrict__ a, const idx_formula &f, uint32_t i) {
    switch (f.kind) {
        case IDX_LINEAR: return f.coef * i + f.intercept;
        case IDX_CYCLE_LINEAR: return (i % f.cycle) * f.coef + f.intercept;
        case IDX_CYCLE_INCREASE: return (i / f.cycle) * f.coef + f.intercept;
        case IDX_RESIDUAL_U8: return f.coef * i + f.intercept + reinterpret_cast<const uint8_t *>(a)[i];
        case IDX_RESIDUAL_U16: return f.coef * i + f.intercept + reinterpret_cast<const uint16_t *>(a)[i];
        case IDX_BRANCH: {
            uint32_t v = f.val[0];
#pragma unroll
            for (int b = 1; b < kIdxBranchMax; b++)
                if ((uint32_t)b < f.n_runs && i >= f.lo[b]) v = f.val[b];
            return v;
        }
        default: return a[i];
    }
}

// a[i] or its formula.  The kernels using formulas instantiate their body twice and pick
// the instantiation once per launch (FX: some formula present), so a plan without
// formulas runs exactly the plain-load code; with FX the kind is a uniform scalar branch.
template <bool FX>
__device__ __forceinline__ uint32_t idx_at(const uint32_t *__restrict__ a, const idx_formula &f, uint32_t i) {
    if constexpr (!FX) return a[i];
    else return f.kind == IDX_ARRAY ? a[i] : idx_eval(a, f, i);
}

// the unit range [a[i], a[i + 1])
template <bool FX>
__device__ __forceinline__ void idx_range(const uint32_t *__restrict__ a, const idx_formula &f, uint32_t i, uint32_t &lo,
                                          uint32_t &hi) {
    if (!FX || f.kind == IDX_ARRAY) {
        lo = a[i];
        hi = a[i + 1];
    } else {
        lo = idx_eval(a, f, i);
        hi = idx_eval(a, f, i + 1);
    }
}
#endif

}  // namespace gsk
