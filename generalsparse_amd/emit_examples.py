"""Emitted programs for the GPU tests.

The reference's code generator writes a plan's arrays and a generated program to
ROOT_PATH_STR/data_source/<id>/ and execute_binary compiles and runs it
(code_generator.cc:633-694, executor.cc:6-104): "./a.out" checks the all-ones known
answer and writes perf_result = "<ms>\\n<GFLOP/s>\\n".  build() calls make() here on the
CPU: it emits one program per plan family below for a fixed seeded matrix and compiles
each with its own make_kernel.sh (hipcc, gfx950), so the GPU tests only run them.
manifest.json lists the program directories (relative to this package)."""
import json
import os
import subprocess
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.path.join(HERE, "emitted")

# (name, pipeline, p0, p1, N, HALF, MODEL_DRIVEN_COMPRESS)
PROGRAMS = [
    ("thread_total_f32", "thread_total", 4, 1, 8, 0, 0),
    ("thread_total_f32_compressed", "thread_total", 4, 1, 8, 0, 1),
    ("warp_segment_f16", "warp_segment", 4, 1, 32, 1, 0),
    ("tblock_warp_total_f16", "tblock_warp_total", 4, 1, 32, 1, 0),
    ("merge_path_f32", "merge_path", 512, 1, 8, 0, 0),
]


def make(jobs=8):
    import shutil
    import generalsparse_amd as gsa
    from generalsparse_amd import datasets as ds
    shutil.rmtree(OUT, ignore_errors=True)
    os.makedirs(OUT, exist_ok=True)
    row, col, val = ds.random_rows(3000, 2000, 12.0, seed=4, empty_frac=0.05)
    manifest = {}
    for name, pipe, p0, p1, N, half, comp in PROGRAMS:
        gsa.set_config("HALF", half)
        gsa.set_config("MODEL_DRIVEN_COMPRESS", comp)
        try:
            plan = gsa.Plan.from_coo(3000, 2000, row, col, val).run_pipeline(pipe, N, p0, p1).compile()
            root = os.path.join(OUT, name)
            os.makedirs(root, exist_ok=True)
            d = plan.generate_program(root, 100)
            manifest[name] = {"dir": os.path.relpath(d, HERE), "N": N, "half": half, "compressed": comp,
                              "pipeline": f"{pipe}({p0},{p1})", "family": plan.info()["kernel_name"]}
            plan.free()
        finally:
            gsa.set_config("HALF", 1)
            gsa.set_config("MODEL_DRIVEN_COMPRESS", 0)

    def build(item):
        name, m = item
        d = os.path.join(HERE, m["dir"])
        r = subprocess.run(["sh", "make_kernel.sh"], cwd=d, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError(f"emitted program {name} does not compile:\n{r.stderr[-4000:]}")
        return name

    with ThreadPoolExecutor(max_workers=jobs) as ex:
        list(ex.map(build, manifest.items()))
    with open(os.path.join(OUT, "manifest.json"), "w") as f:
        json.dump(manifest, f, indent=1)
    return manifest


if __name__ == "__main__":
    print(json.dumps(make(), indent=1))
