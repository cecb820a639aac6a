"""CPU: the C-ABI library loads, exports every symbol declared in include/ofdmsync.h, and
rejects bad arguments before touching the GPU.  No compute calls (no GPU here)."""
import ctypes
import os
import re

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "ofdmsync.h")
LIB = os.path.join(ROOT, "ofdm-sync-math_amd", "ofdm_sync_amd", "libofdmsync.so")


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import __graft_entry__ as g
        g.build_hip()
    return ctypes.CDLL(LIB)


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(ofs_\w+)\s*\(", txt, re.M)))


def test_header_declares_the_boundary():
    syms = declared_symbols()
    assert {"ofs_aa_detect", "ofs_sc_metric", "ofs_minn_metric", "ofs_minn_rtl",
            "ofs_minn_rtl_gate", "ofs_cp_cfo", "ofs_version", "ofs_status_string"} <= set(syms)


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s


def test_exports_are_c_linkage():
    out = os.popen(f"nm -D --defined-only {LIB}").read()
    exported = set(re.findall(r"\bT\s+(ofs_\w+)$", out, re.M))
    assert set(declared_symbols()) <= exported


def test_version_and_status(lib):
    lib.ofs_version.restype = ctypes.c_int32
    assert lib.ofs_version() >= 100
    lib.ofs_status_string.restype = ctypes.c_char_p
    lib.ofs_status_string.argtypes = [ctypes.c_int32]
    assert lib.ofs_status_string(0) == b"ok"
    assert b"invalid" in lib.ofs_status_string(-1)


def test_argument_validation_without_gpu(lib):
    """Bad arguments return OFS_EINVAL (-1) before any HIP call."""
    from ofdm_sync_amd import _lib as L
    L._declare(lib)
    # null input
    assert lib.ofs_aa_detect(0, None, 1, 1, 16, 4, 0, None, None, None, None, 0, 0.1, 1, 1.0, 0,
                             None, None, None, None) == -1
    # bad format / precision
    assert lib.ofs_aa_detect(7, 1, 1, 1, 16, 4, 0, None, None, None, None, 0, 0.1, 1, 1.0, 0,
                             None, None, None, None) == -1
    assert lib.ofs_sc_metric(0, 1, 1, 1, 16, 8, 0, 9, None, None, None, None) == -1
    # odd S&C symbol length
    assert lib.ofs_sc_metric(0, 1, 1, 1, 16, 7, 0, 0, None, None, None, None) == -1
    # detect requested without event buffers
    assert lib.ofs_aa_detect(0, 1, 1, 1, 16, 4, 0, None, None, None, None, 1, 0.1, 1, 1.0, 4,
                             None, None, None, None) == -1
    # minn_rtl without required outputs / bad Q
    assert lib.ofs_minn_rtl(0, 1, 1, 1, 16, 4, 3, 0, 3276, 15, None, None, None, None, None, None,
                            None, None, 0, 2, 0, 0, None, None, None, None) == -1
    assert lib.ofs_minn_rtl(0, 1, 1, 1, 16, 0, 3, 0, 3276, 15, 1, None, None, 1, None, None,
                            None, None, 0, 2, 0, 0, None, None, None, None) == -1
    assert lib.ofs_cp_cfo(0, 1, 1, 1, 16, None, 8, 4, 1.0, None, None, None) == -1
    # cp search: null est, zero window, bad mode
    assert lib.ofs_cp_search(0, 1, 1, 1, 16, None, 8, 4, 2, 0, 1.0, None, None, 1, 1, None) == -1
    assert lib.ofs_cp_search(0, 1, 1, 1, 16, 1, 8, 0, 2, 0, 1.0, None, None, 1, 1, None) == -1
    assert lib.ofs_cp_search(0, 1, 1, 1, 16, 1, 8, 4, 2, 5, 1.0, None, None, 1, 1, None) == -1
    assert lib.ofs_minn_rtl_gate(None, None, None, 1, 16, 2, 0, 1, None, None, None, None) == -1
    # receiver back-end: N not a power of two, n_used > N, missing starts
    bk = (0, 1, 1, 1, 64)
    assert lib.ofs_rx_backend(*bk, 48, 8, 1.0, 1, 1, None, 8, 1, 1, 0, 1, 0, *([None] * 8), None) == -1
    assert lib.ofs_rx_backend(*bk, 32, 8, 1.0, 1, 1, None, 40, 1, 1, 0, 1, 0, *([None] * 8), None) == -1
    assert lib.ofs_rx_backend(*bk, 32, 8, 1.0, None, 1, None, 8, 1, 1, 0, 1, 0, *([None] * 8), None) == -1
    # synthesis: null base, bad output format, non-positive sample rate
    assert lib.ofs_synth_batch(None, 8, 1, 1, 8, 0, 0.0, 1.0, 0.0, 0.0, 1.0, 1, 0, 1.0, 1, None, None) == -1
    assert lib.ofs_synth_batch(1, 8, 1, 1, 8, 0, 0.0, 1.0, 0.0, 0.0, 1.0, 1, 9, 1.0, 1, None, None) == -1
    assert lib.ofs_synth_batch(1, 8, 1, 1, 8, 0, 0.0, 1.0, 0.0, 0.0, 0.0, 1, 0, 1.0, 1, None, None) == -1
    # empty batches are valid no-ops
    assert lib.ofs_sc_metric(0, 1, 0, 1, 16, 8, 0, 0, None, None, None, None) == 0
    assert lib.ofs_minn_metric(0, 1, 1, 1, 4, 8, 0, None, None, None, None) == 0
    # ... and their pointers may be NULL (no data behind them): B = 0 with every array null
    assert lib.ofs_aa_detect(0, None, 0, 1, 1024, 512, 0, None, None, None, None, 1, 0.15, 128, 15.36e6, 4,
                             None, None, None, None) == 0
    assert lib.ofs_sc_metric(0, None, 0, 1, 4096, 2048, 1, 0, None, None, None, None) == 0
    assert lib.ofs_sc_minn_metric(0, None, 0, 1, 4096, 2048, 0, None, None, None, None, None, None, None) == 0
    assert lib.ofs_minn_rtl(2, None, 0, 1, 1024, 64, 3, 0, 3276, 15, None, None, None, None, None, None,
                            None, None, 1, 2, 0, 4, None, None, None, None) == 0
    assert lib.ofs_cp_cfo(0, None, 0, 1, 16, None, 8, 4, 1.0, None, None, None) == 0
    assert lib.ofs_trailing_average(1, None, 0, 100, 8, 0, None, None) == 0
    # zc_freq partial sums: branch group outside the branch count, > 4 branches or > 64 bins per group,
    # null output; the finish kernel: bad precision; a too-short stream is OFS_ESHORT (-4)
    ib = (ctypes.c_int32 * 2)(1, -1)
    tb = (ctypes.c_double * 4)(1.0, 0.0, 1.0, 0.0)
    assert lib.ofs_zc_freq_partial(0, 1, 1, 2, 100, 1, 2, 16, 0, 2, ib, tb, 0, 1, None) == -1
    assert lib.ofs_zc_freq_partial(0, 1, 1, 6, 100, 0, 5, 16, 0, 2, ib, tb, 0, 1, None) == -1
    assert lib.ofs_zc_freq_partial(0, 1, 1, 1, 100, 0, 1, 16, 0, 65, ib, tb, 0, 1, None) == -1
    assert lib.ofs_zc_freq_partial(0, 1, 1, 1, 100, 0, 1, 16, 0, 2, ib, tb, 0, None, None) == -1
    assert lib.ofs_zc_freq_partial(0, 1, 1, 1, 10, 0, 1, 16, 0, 2, ib, tb, 0, 1, None) == -4
    assert lib.ofs_zc_freq_finish(1, 1, 10, 1.0, 7, 1, None) == -1
    assert lib.ofs_zc_freq_finish(None, 0, 10, 1.0, 0, None, None) == 0
    # a null pointer for a NON-empty buffer is still refused
    assert lib.ofs_aa_detect(0, None, 1, 1, 1024, 512, 0, None, None, None, None, 0, 0.15, 128, 15.36e6, 0,
                             None, None, None, None) == -1


def test_product_path_refuses_cpu():
    """No CPU fallback: the drop-in raises when no GPU is present."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from ofdm_sync_amd import sync_aa
    with pytest.raises(RuntimeError, match="GPU"):
        sync_aa.aa_detect_streaming([1 + 1j] * 32, L=4)


def test_library_reads_no_environment():
    """Dispatch and arithmetic depend only on the call's arguments (and on debug variants set
    through ofs_debug_set_variant): no source of the shipped library calls getenv / secure_getenv."""
    csrc = os.path.join(ROOT, "ofdm-sync-math_amd", "csrc")
    for f in sorted(os.listdir(csrc)):
        txt = open(os.path.join(csrc, f)).read()
        assert not re.search(r"\b(secure_)?getenv\s*\(", txt), f
    out = os.popen(f"nm -D --undefined-only {LIB}").read()
    assert not re.search(r"\bU\s+(secure_)?getenv\b", out)


def test_debug_variants_entry_point(lib):
    """ofs_debug_set_variant / _get_variant / _reset_variants: unknown names refused, values
    round-trip, reset clears every variant, and the default is unset."""
    from ofdm_sync_amd import _lib as L
    L._declare(lib)
    unset = -(1 << 63)
    assert lib.ofs_debug_reset_variants() == 0
    hdr = open(HEADER).read()
    block = hdr[hdr.index("Names (value meaning):"):hdr.index("ofs_debug_set_variant returns")]
    names = re.findall(r"^ \*   ([A-Z][A-Z0-9_]+)\s", block, re.M)
    assert {"EXACT", "MC_FUSED", "ZS_PAIR", "FAST_SCAN", "BE_FAST", "ZC_SEQ"} <= set(names)
    for n in names:
        assert lib.ofs_debug_get_variant(n.encode()) == unset, n
        assert lib.ofs_debug_set_variant(n.encode(), 7) == 0, n
        assert lib.ofs_debug_get_variant(n.encode()) == 7, n
    assert lib.ofs_debug_set_variant(b"NO_SUCH_KNOB", 1) == -1
    assert lib.ofs_debug_get_variant(b"NO_SUCH_KNOB") == unset
    assert lib.ofs_debug_set_variant(b"EXACT", unset) == 0 and lib.ofs_debug_get_variant(b"EXACT") == unset
    assert lib.ofs_debug_reset_variants() == 0
    assert all(lib.ofs_debug_get_variant(n.encode()) == unset for n in names)


def test_debug_variants_are_per_thread(lib):
    """The variant table is thread_local: a variant forced by one thread (a test) is not seen by
    calls another thread makes, and a new thread starts with every variant unset."""
    import threading
    from ofdm_sync_amd import _lib as L
    L._declare(lib)
    unset = -(1 << 63)
    assert lib.ofs_debug_set_variant(b"EXACT", 0) == 0
    seen = {}

    def other():
        seen["before"] = lib.ofs_debug_get_variant(b"EXACT")
        lib.ofs_debug_set_variant(b"ZS_PAIR", 5)
        seen["own"] = lib.ofs_debug_get_variant(b"ZS_PAIR")
    t = threading.Thread(target=other)
    t.start()
    t.join()
    assert seen == {"before": unset, "own": 5}
    assert lib.ofs_debug_get_variant(b"EXACT") == 0
    assert lib.ofs_debug_get_variant(b"ZS_PAIR") == unset
    assert lib.ofs_debug_reset_variants() == 0


def test_product_mirror_reads_no_environment():
    """The Python mirror takes no switch from the environment: OFS_LIB (or any other variable)
    cannot swap the library or skip its source-hash check."""
    pkg = os.path.join(ROOT, "ofdm-sync-math_amd", "ofdm_sync_amd")
    for f in sorted(os.listdir(pkg)):
        if f.endswith(".py"):
            txt = open(os.path.join(pkg, f)).read()
            # shard.py reads the torch.distributed launch contract (RANK / WORLD_SIZE / LOCAL_RANK) only
            names = set(re.findall(r"os\.environ\.get\(\"(\w+)\"", txt))
            assert names <= ({"RANK", "WORLD_SIZE", "LOCAL_RANK"} if f == "shard.py" else set()), (f, names)
            assert not re.search(r"os\.environ\[|getenv\s*\(", txt), f
            assert len(re.findall(r"os\.environ", txt)) == len(re.findall(r"os\.environ\.get\(\"", txt)), f


def test_library_path_ignores_ofs_lib_and_tuning_loader_refuses_product_build(tmp_path):
    """In a fresh process with OFS_LIB pointing elsewhere, the mirror still loads the in-tree
    library (hash-checked); use_tuning_library accepts only a tools/variants.py build (baked hash
    variant-<name>), so it refuses the product library itself."""
    import subprocess
    import sys
    if not os.path.exists(LIB):
        import __graft_entry__ as g
        g.build_hip()
    code = (
        "import sys; sys.path.insert(0, %r)\n"
        "from ofdm_sync_amd import _lib\n"
        "l = _lib.lib(); import os\n"
        "assert os.path.samefile(l._name, %r), l._name\n"
        "_lib._lib = None\n"
        "try:\n"
        "    _lib.use_tuning_library(%r)\n"
        "except ImportError as e:\n"
        "    print('refused', e)\n"
        "else:\n"
        "    raise SystemExit('accepted')\n"
    ) % (os.path.join(ROOT, "ofdm-sync-math_amd"), LIB, LIB)
    env = dict(os.environ, OFS_LIB=str(tmp_path / "nonexistent.so"))
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr + r.stdout
    assert "refused" in r.stdout
