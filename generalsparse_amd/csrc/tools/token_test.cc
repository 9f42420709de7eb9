// token_test <mtx> <N> [pipeline] [p0] [p1] -- the reference's CLI entry
// (token_test.cc:1625-1847) on the MI355X engine.
//
// Like the reference: DENSE_MATRIX_SIZE := N, the .mtx is read with every value
// set to 1 (struct.cc:186-200), the pipeline (default thread_total(4,1), the
// one main() runs) lowers it to a plan, the code generator writes the plan and a
// generated program into ROOT_PATH_STR/data_source/<id>/.  Instead of shelling
// out to compile that program (executor.cc:60-104), the plan runs in-process on
// the GPU; the result is checked against C[i][j] = nnz(row i) (the reference's
// all-ones known answer) and "<ms for repeat launches>\n<GFLOP/s>\n" is written
// to perf_result (code_generator.cc:643-648).  --exec-program additionally
// builds and runs the generated program (hipcc) like execute_binary.
#include "../../../include/generalsparse.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                 \
    do {                                                                      \
        int rc_ = (x);                                                        \
        if (rc_ != 0) {                                                       \
            std::fprintf(stderr, "%s failed (%d): %s\n", #x, rc_, gs_last_error()); \
            return 1;                                                         \
        }                                                                     \
    } while (0)

#define HK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));         \
            return 1;                                                                   \
        }                                                                               \
    } while (0)

int main(int argc, char **argv) {
    if (argc < 3) {
        std::fprintf(stderr, "usage: token_test <matrix.mtx> <N> [pipeline] [p0] [p1] [--f32] [--exec-program]\n");
        return 2;
    }
    std::string mtx = argv[1];
    int N = std::atoi(argv[2]);
    std::string pipeline = argc > 3 && argv[3][0] != '-' ? argv[3] : "thread_total";
    int p0 = argc > 4 && argv[4][0] != '-' ? std::atoi(argv[4]) : 4;
    int p1 = argc > 5 && argv[5][0] != '-' ? std::atoi(argv[5]) : 1;
    bool f32 = false, exec_prog = false;
    for (int i = 3; i < argc; i++) {
        if (!std::strcmp(argv[i], "--f32")) f32 = true;
        if (!std::strcmp(argv[i], "--exec-program")) exec_prog = true;
    }
    const char *root_env = std::getenv("GS_ROOT_PATH");
    std::string root = root_env ? root_env : ".";
    const int repeat = 10000;  // generate_final_program(10000), token_test.cc:1081

    gs_plan_t *plan = nullptr;
    CK(gs_plan_create_from_mtx(mtx.c_str(), 1, &plan));
    CK(gs_set_config_int("HALF", f32 ? 0 : 1));
    CK(gs_plan_run_pipeline(plan, pipeline.c_str(), N, p0, p1));
    CK(gs_plan_compile(plan));
    char dir[4096] = {0};
    CK(gs_plan_generate_program(plan, root.c_str(), 100, dir, sizeof(dir)));
    std::vector<char> log(1 << 16);
    gs_plan_log(plan, log.data(), (int)log.size());
    std::printf("%s", log.data());
    CK(gs_plan_upload(plan, f32 ? GS_F32 : GS_F16, 0));
    gs_plan_info info;
    CK(gs_plan_info_get(plan, &info));
    std::printf("plan: %s rows=%llu cols=%llu nnz=%llu stored=%llu units=%llu\n", info.kernel_name,
                (unsigned long long)info.rows, (unsigned long long)info.cols, (unsigned long long)info.nnz,
                (unsigned long long)info.nnz_stored, (unsigned long long)info.n_units);

    const size_t es = f32 ? 4 : 2;
    std::vector<uint16_t> hB16(info.cols * N, 0x3c00);  // fp16 1.0
    std::vector<float> hB32(info.cols * N, 1.0f);
    void *dB = nullptr, *dC = nullptr;
    HK(hipMalloc(&dB, info.cols * N * es));
    HK(hipMalloc(&dC, info.rows * N * es));
    HK(hipMemcpy(dB, f32 ? (void *)hB32.data() : (void *)hB16.data(), info.cols * N * es, hipMemcpyHostToDevice));
    CK(gs_spmm(plan, dB, dC, N, nullptr));
    HK(hipDeviceSynchronize());
    // known answer: C[i][j] = nnz(row i)
    std::vector<uint64_t> row(info.nnz);
    std::vector<uint64_t> nnz_row(info.rows, 0);
    {
        // recount from the file's rows: re-read via a fresh plan's arrays
        gs_plan_t *raw = nullptr;
        CK(gs_plan_create_from_mtx(mtx.c_str(), 1, &raw));
        CK(gs_plan_array_read_u64(raw, "GLOBAL_META_nz_row_indices_0", row.data(), row.size()));
        gs_plan_free(raw);
        for (uint64_t r : row) nnz_row[r]++;
    }
    std::vector<float> out(info.rows * N);
    if (f32) {
        HK(hipMemcpy(out.data(), dC, out.size() * 4, hipMemcpyDeviceToHost));
    } else {
        std::vector<_Float16> h(info.rows * N);
        HK(hipMemcpy(h.data(), dC, h.size() * 2, hipMemcpyDeviceToHost));
        for (size_t i = 0; i < h.size(); i++) out[i] = (float)h[i];
    }
    long wrong = 0;
    for (uint64_t i = 0; i < info.rows; i++)
        for (int j = 0; j < N; j++)
            if (out[i * N + j] != (float)(_Float16)(float)nnz_row[i] && out[i * N + j] != (float)nnz_row[i]) {
                if (wrong < 10)
                    std::printf("Wrong result: i = %llu, j = %d, result = %f, reference = %f.\n",
                                (unsigned long long)i, j, out[i * N + j], (double)nnz_row[i]);
                wrong++;
            }
    std::printf("wrong number:%ld\n", wrong);
    if (!wrong) std::printf("correct\n");
    hipEvent_t e0, e1;
    HK(hipEventCreate(&e0));
    HK(hipEventCreate(&e1));
    HK(hipEventRecord(e0, nullptr));
    for (int i = 0; i < repeat; i++) CK(gs_spmm(plan, dB, dC, N, nullptr));
    HK(hipEventRecord(e1, nullptr));
    HK(hipEventSynchronize(e1));
    float ms = 0;
    HK(hipEventElapsedTime(&ms, e0, e1));
    HK(hipEventDestroy(e0));
    HK(hipEventDestroy(e1));
    double gflops = 2.0 * (double)info.nnz * N * repeat / (ms * 1e-3) / 1e9;  // padding excluded
    std::string pr = std::string(dir) + "/perf_result";
    if (FILE *f = std::fopen(pr.c_str(), "w")) {
        std::fprintf(f, "%f\n%f\n", ms, gflops);
        std::fclose(f);
    }
    std::printf("%s %f\n", mtx.c_str(), gflops);
    std::printf("%s : min time: %f\n", mtx.c_str(), ms / repeat);
    if (exec_prog) {
        std::string cmd = "cd " + std::string(dir) + " && sh make_kernel.sh > compile_result 2>&1 && ./a.out " + mtx +
                          " " + std::to_string(N);
        int rc = std::system(cmd.c_str());
        std::printf("generated program exit code %d\n", rc);
        if (rc != 0) wrong = wrong ? wrong : -1;
    }
    HK(hipFree(dB));
    HK(hipFree(dC));
    gs_plan_free(plan);
    return wrong ? 1 : 0;
}
