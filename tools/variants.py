"""Build tuning variants of libofdmsync.so: only the translation units whose flags change are
recompiled per variant; the others are compiled once.  Diagnostic tooling (not the product).

    python tools/variants.py aa_fast.hip "pd2=-DOFS_STREAM_PD=2" "w4=-DOFS_STREAM_WAVES=4" ...
Writes build/libofdmsync_<name>.so (source-hash check is skipped for OFS_LIB builds).
"""
import concurrent.futures as cf
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "ofdm-sync-math_amd", "csrc")
OUT = os.path.join(ROOT, "build")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-fPIC", "-I" + os.path.join(ROOT, "include")]
LIBS = ["-L/opt/rocm/lib", "-lrocfft", "-Wl,-rpath,/opt/rocm/lib"]


def cc(src, obj, extra):
    subprocess.run(["/opt/rocm/bin/hipcc", *FLAGS, *extra, "-c", src, "-o", obj], check=True)
    return obj


def main():
    tu, variants = sys.argv[1], sys.argv[2:]
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    with cf.ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        base = {s: ex.submit(cc, os.path.join(CSRC, s), os.path.join(OUT, s + ".o"), []) for s in srcs if s != tu}
        var = {}
        for v in variants:
            name, _, fl = v.partition("=")
            var[name] = ex.submit(cc, os.path.join(CSRC, tu), os.path.join(OUT, f"{tu}.{name}.o"), fl.split())
        objs = [f.result() for f in base.values()]
        for name, f in var.items():
            so = os.path.join(OUT, f"libofdmsync_{name}.so")
            subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-shared", "-fPIC", "-o", so,
                            *objs, f.result(), *LIBS], check=True)
            print(so)


if __name__ == "__main__":
    main()
