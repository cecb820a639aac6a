"""Build tuning variants of libofdmsync.so: only the translation units whose flags change are
recompiled per variant; the others are compiled once.  Diagnostic tooling (not the product).

    python tools/variants.py aa_fast.hip "pd2=-DOFS_STREAM_PD=2" "w4=-DOFS_STREAM_WAVES=4" ...
Writes build/libofdmsync_<name>.so (load one with `OFS_LIB=... python tools/<tool>.py`: the tools pass it to
_lib.use_tuning_library, which accepts only a library whose baked hash reads variant-<name>).
"""
import concurrent.futures as cf
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import __graft_entry__ as G  # noqa: E402

CSRC = G.CSRC
OUT = os.path.join(ROOT, "build")


def main():
    tu, variants = sys.argv[1], sys.argv[2:]
    os.makedirs(OUT, exist_ok=True)
    srcs = sorted(f for f in os.listdir(CSRC) if f.endswith(".hip"))
    with cf.ThreadPoolExecutor(min(16, os.cpu_count() or 1)) as ex:
        base = [ex.submit(G.compile_cached, os.path.join(CSRC, s)) for s in srcs if s != tu]
        var = {}
        for v in variants:
            name, _, fl = v.partition("=")
            var[name] = ex.submit(G.compile_cached, os.path.join(CSRC, tu), fl.split())
        objs = [f.result() for f in base]
        for name, f in var.items():
            so = os.path.join(OUT, f"libofdmsync_{name}.so")
            G.link_lib([*objs, f.result()], so, "variant-" + name)
            print(so)
    G.build_hip()       # keep the in-tree library in step with the sources (tests load it unbuilt)


if __name__ == "__main__":
    main()
