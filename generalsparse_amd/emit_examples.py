"""Emitted programs for the GPU tests.

The reference's code generator writes a plan's arrays and a generated program to
ROOT_PATH_STR/data_source/<id>/ and execute_binary compiles and runs it
(code_generator.cc:633-694, executor.cc:6-104): "./a.out" checks the all-ones known
answer and writes perf_result = "<ms>\\n<GFLOP/s>\\n".  build() calls make() here on the
CPU: it emits one program per plan below and compiles each with its own make_kernel.sh
(hipcc, gfx950), so the GPU tests only run them.  The fp16 block-row and 2:4 plans emit the
matrix-core kernels gs_spmm launches (k_mfma_rows, k_mfma_ks, k_nm_mfma: the layout arrays
as binary sidecars next to the plan's text arrays).

The full-size C2 programs and the 2:4 program ("regen") are compiled here, then their ~170 MB of plan arrays
are deleted so they do not travel with every GPU call: the GPU test re-emits the arrays
from the same seeded matrix on the box (plan.generate_program), checks the re-emitted
kernel_file.hip is byte-identical to the compiled one, and runs the prebuilt a.out there.
manifest.json lists the program directories (relative to this package)."""
import json
import os
import shutil
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "emitted")

# (name, matrix, pipeline, p0, p1, N, HALF, MODEL_DRIVEN_COMPRESS, regen)
PROGRAMS = [
    ("thread_total_f32", "random", "thread_total", 4, 1, 8, 0, 0, False),
    ("thread_total_f32_compressed", "random", "thread_total", 4, 1, 8, 0, 1, False),
    ("warp_segment_f16", "random", "warp_segment", 4, 1, 32, 1, 0, False),
    ("tblock_warp_total_f16", "random", "tblock_warp_total", 4, 1, 32, 1, 0, False),
    ("merge_path_f32", "random", "merge_path", 512, 1, 8, 0, 0, False),
    # the matrix-core kernels on small matrices (shipped whole), and C3's plan on 2,048 rows
    ("mfma_rows_f16", "pruned", "block_total", 20, 1, 32, 1, 0, False),
    ("mfma_ks_f16", "pruned", "block_total", 64, 1, 32, 1, 0, False),
    ("nm_mfma_f16_n128", "two_four", "col_direction_nm", 32, 1, 128, 1, 0, True),
    # the C2 plans at full size (BASELINE configs[1]; arrays re-emitted on the GPU box)
    ("c2_tblock_warp_total_20_2", "c2", "tblock_warp_total", 20, 2, 32, 1, 0, True),
    ("c2_block_total_80", "c2", "block_total", 80, 1, 32, 1, 0, True),
]


def matrix(kind):
    from generalsparse_amd import datasets as ds
    if kind == "random":
        return (3000, 2000) + ds.random_rows(3000, 2000, 12.0, seed=4, empty_frac=0.05)
    if kind == "pruned":
        return (400, 2000) + ds.pruned_weight(400, 2000, 0.7, 17)
    if kind == "two_four":  # C3's plan (col_direction_nm on 2:4 rows) on 2,048 of its 28,672 rows
        return (2048, 7168) + ds.two_four(2048, 7168, 30)
    if kind == "c2":
        return (5120, 5120) + ds.pruned_weight(5120, 5120, 0.7, 13)
    raise ValueError(kind)


def emit(name, kind, pipe, p0, p1, N, half, comp, root):
    """emits one program under root; returns its directory"""
    import generalsparse_amd as gsa
    M, K, row, col, val = matrix(kind)
    gsa.set_config("HALF", half)
    gsa.set_config("MODEL_DRIVEN_COMPRESS", comp)
    try:
        plan = gsa.Plan.from_coo(M, K, row, col, val).run_pipeline(pipe, N, p0, p1).compile()
        os.makedirs(root, exist_ok=True)
        d = plan.generate_program(root, 100)
        plan.free()
        return d
    finally:
        gsa.set_config("HALF", 1)
        gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)


def device_kernel(d):
    """the kernel a generated program launches (from its source)"""
    src = open(os.path.join(d, "kernel_file.hip")).read()
    for k in ("k_mfma_ks", "k_mfma_rows", "k_nm_mfma", "k_thread_total", "k_warp_rows", "k_block_rows",
              "k_bitmap_segment", "k_row_chunks", "k_merge_rows", "k_merge_path"):
        if f"gsk::{k}<" in src:
            return k
    return "?"


def make(jobs=8):
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(OUT, exist_ok=True)
    manifest = {}
    for name, kind, pipe, p0, p1, N, half, comp, regen in PROGRAMS:
        d = emit(name, kind, pipe, p0, p1, N, half, comp, os.path.join(OUT, name))
        manifest[name] = {"dir": os.path.relpath(d, HERE), "N": N, "half": half, "compressed": comp,
                          "matrix": kind, "pipeline": pipe, "p0": p0, "p1": p1, "regen": regen,
                          "kernel": device_kernel(d)}

    def build(item):
        name, m = item
        d = os.path.join(HERE, m["dir"])
        r = subprocess.run(["sh", "make_kernel.sh"], cwd=d, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"emitted program {name} does not compile:\n{r.stderr[-4000:]}")
        if m["regen"]:  # keep the program, drop the plan arrays (re-emitted on the GPU box)
            for f in os.listdir(d):
                if f.endswith("_0") or f.endswith("_0.bin"):
                    os.remove(os.path.join(d, f))
        return name

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(build, manifest.items()))
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    return manifest


if __name__ == "__main__":
    print(json.dumps(make(), indent=1))
