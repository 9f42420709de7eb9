// Probe: operand layout and issue cost of v_smfmac_f32_16x16x64_f16 on gfx950.
// Hypothesis tested: lane l holds row/col (l%16) and the dense k-range
// [16*(l/16), 16*(l/16)+16) of the 64-wide step; A's 8 compressed halfs are
// pairs per 4-wide group (value i in group i/2), idx bits [2i+1:2i] = position
// of value i in its group; B's 16 halfs are the 16 dense k of that range.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <cmath>
#include <vector>
typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h16 __attribute__((ext_vector_type(16)));
typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void k_one(const h8 *a, const h16 *b, const int *idx, f4 *c, int hi) {
    int l = threadIdx.x;
    f4 acc = {0, 0, 0, 0};
    if (hi) acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a[l], b[l], acc, idx[l], 0, 1);
    else acc = __builtin_amdgcn_smfmac_f32_16x16x64_f16(a[l], b[l], acc, idx[l], 0, 0);
    c[l] = acc;
}

__global__ void k_rate(const h8 *a, const h16 *b, const int *idx, f4 *c, long long *t, int iters) {
    int l = threadIdx.x;
    h8 av = a[l]; h16 bv = b[l]; int ix = idx[l];
    f4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    long long t0 = clock64();
    for (int i = 0; i < iters; i++) {
        c0 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, c0, ix, 0, 0);
        c1 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, c1, ix, 0, 0);
        c2 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, c2, ix, 0, 0);
        c3 = __builtin_amdgcn_smfmac_f32_16x16x64_f16(av, bv, c3, ix, 0, 0);
    }
    long long t1 = clock64();
    c[l] = c0 + c1 + c2 + c3;
    if (l == 0) t[0] = t1 - t0;
}

int main() {
    srand(7);
    std::vector<_Float16> A(64 * 8), B(64 * 16);
    std::vector<int> I(64);
    std::vector<float> Ad(64 * 16, 0.f);  // lane-dense expansion
    for (int l = 0; l < 64; l++) {
        unsigned ix = 0;
        for (int g = 0; g < 4; g++) {
            int p0 = rand() % 4, p1 = rand() % 4;
            while (p1 == p0) p1 = rand() % 4;
            if (p0 > p1) { int t = p0; p0 = p1; p1 = t; }
            float v0 = (float)(rand() % 7 - 3), v1 = (float)(rand() % 7 - 3);
            A[l * 8 + 2 * g] = (_Float16)v0; A[l * 8 + 2 * g + 1] = (_Float16)v1;
            ix |= (unsigned)p0 << (4 * g); ix |= (unsigned)p1 << (4 * g + 2);
            Ad[l * 16 + 4 * g + p0] = v0; Ad[l * 16 + 4 * g + p1] = v1;
        }
        I[l] = (int)ix;
        for (int e = 0; e < 16; e++) B[l * 16 + e] = (_Float16)(float)(rand() % 5 - 2);
    }
    h8 *da; h16 *db; int *di; f4 *dc; long long *dt;
    hipMalloc(&da, 64 * 16); hipMalloc(&db, 64 * 32); hipMalloc(&di, 256); hipMalloc(&dc, 64 * 16); hipMalloc(&dt, 8);
    hipMemcpy(da, A.data(), 64 * 16, hipMemcpyHostToDevice);
    hipMemcpy(db, B.data(), 64 * 32, hipMemcpyHostToDevice);
    for (int hi = 0; hi < 2; hi++) {
        std::vector<int> Ii(64);
        for (int l = 0; l < 64; l++) Ii[l] = hi ? (I[l] << 16) | 0x1b1b : I[l] | (0x4e4e << 16);
        hipMemcpy(di, Ii.data(), 256, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, da, db, di, dc, hi);
        std::vector<float> C(64 * 4);
        hipMemcpy(C.data(), dc, 64 * 16, hipMemcpyDeviceToHost);
        // accumulator layout of 16x16 MFMA: lane l holds column l%16, rows 4*(l/16)+i
        double maxerr = 0;
        for (int l = 0; l < 64; l++)
            for (int i = 0; i < 4; i++) {
                int n = l % 16, m = 4 * (l / 16) + i;
                double ref = 0;
                for (int g = 0; g < 4; g++)
                    for (int p = 0; p < 16; p++) ref += Ad[(m + 16 * g) * 16 + p] * (float)B[(n + 16 * g) * 16 + p];
                maxerr = fmax(maxerr, fabs(ref - C[l * 4 + i]));
            }
        printf("abid=%d hypothesis max|err| = %g %s\n", hi, maxerr, maxerr == 0 ? "MATCH" : "mismatch");
    }
    for (int iters : {1000, 4000}) {
        hipLaunchKernelGGL(k_rate, dim3(1), dim3(64), 0, 0, da, db, di, dc, dt, iters);
        long long t; hipMemcpy(&t, dt, 8, hipMemcpyDeviceToHost);
        printf("iters %d: %.2f cycles per smfmac (clock64 units)\n", iters, (double)t / (4.0 * iters));
    }

    // pairing map: A = a single 1 at row 0, lane group g, dense position p (idx puts
    // value 0 of group p/4 at p%4); B element e of lane (n + 16*gb) = 1 + e + 16*gb for
    // column n = 0 only -> C[0][0] names the B element the A position meets
    {
        std::vector<_Float16> B1(64 * 16, (_Float16)0.f);
        for (int gb = 0; gb < 4; gb++)
            for (int e = 0; e < 16; e++) B1[(16 * gb) * 16 + e] = (_Float16)(float)(1 + e + 16 * gb);
        hipMemcpy(db, B1.data(), 64 * 32, hipMemcpyHostToDevice);
        printf("pairing (A lane group g, dense pos p) -> B id (1 + e + 16*gb):\n");
        for (int g = 0; g < 4; g++) {
            printf("g%d:", g);
            for (int p = 0; p < 16; p++) {
                std::vector<_Float16> A1(64 * 8, (_Float16)0.f);
                std::vector<int> I1(64, 0x4444);  // positions 0,1 in every group
                int grp = p / 4, pos = p % 4;
                int other = pos == 0 ? 1 : 0;
                int lo = pos < other ? pos : other, hi2 = pos < other ? other : pos;
                unsigned ix = 0x4444u & ~(0xfu << (4 * grp));
                ix |= (unsigned)lo << (4 * grp); ix |= (unsigned)hi2 << (4 * grp + 2);
                I1[16 * g] = (int)ix;
                A1[(16 * g) * 8 + 2 * grp + (pos == lo ? 0 : 1)] = (_Float16)1.f;
                hipMemcpy(da, A1.data(), 64 * 16, hipMemcpyHostToDevice);
                hipMemcpy(di, I1.data(), 256, hipMemcpyHostToDevice);
                hipLaunchKernelGGL(k_one, dim3(1), dim3(64), 0, 0, da, db, di, dc, 0);
                std::vector<float> C(64 * 4);
                hipMemcpy(C.data(), dc, 64 * 16, hipMemcpyDeviceToHost);
                printf(" %3.0f", C[0]);
            }
            printf("\n");
        }
    }
    return 0;
}
