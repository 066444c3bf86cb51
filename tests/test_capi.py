"""CPU-side checks of the C ABI: the library loads and exports every symbol include/nfdpf.h
declares; argument validation rejects bad calls before any launch (no GPU needed)."""
import ctypes
import os
import re

import pytest

from _util import ROOT

HEADER = os.path.join(ROOT, "include", "nfdpf.h")


def declared_symbols():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"NFDPF_API\s+[\w\s\*]+?\b(nfdpf_\w+)\s*\(", txt)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ("nfdpf_cond_stack", "nfdpf_maf_stack", "nfdpf_soft_resample", "nfdpf_ot_resample",
              "nfdpf_filter_step", "nfdpf_measurement", "nfdpf_normalize_log_probs", "nfdpf_ess_gate",
              "nfdpf_particle_init", "nfdpf_ot_workspace_bytes", "nfdpf_version", "nfdpf_last_error"):
        assert s in syms


def test_library_exports_every_declared_symbol():
    from nfdpf import _lib
    lib = _lib.load()
    for s in declared_symbols():
        assert hasattr(lib, s), s
        assert s in _lib.SIGNATURES, f"{s} has no ctypes signature"
    assert lib.nfdpf_version() >= 1


def test_no_stray_exports():
    out = os.popen(f"nm -D --defined-only {os.path.join(ROOT, 'normalizing-flows-dpfs_amd', 'libnfdpf.so')}").read()
    exported = {l.split()[-1] for l in out.splitlines() if " T " in l}
    assert exported == set(declared_symbols()), exported ^ set(declared_symbols())


def test_filter_desc_layout_matches_header():
    """ctypes mirror of nfdpf_filter_desc: same field names in the same order as the header."""
    from nfdpf._lib import FilterDesc
    body = open(HEADER).read().split("typedef struct nfdpf_filter_desc {")[1].split("} nfdpf_filter_desc;")[0]
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    names = []
    for decl in body.split(";"):
        decl = decl.strip()
        if not decl:
            continue
        decl = re.sub(r"^(const\s+)?\w+\s*", "", decl)
        names += [n.strip().lstrip("*").strip() for n in decl.split(",")]
    assert [f[0] for f in FilterDesc._fields_] == names


def test_argument_validation_without_device():
    from nfdpf import _lib
    lib = _lib.load()
    # null pointers -> EINVAL, message set, nothing launched
    rc = lib.nfdpf_cond_stack(None, 2, 2, 4, 8, None, None, 10, 1, 0, 0.0, 1.0, None, None, None, None)
    assert rc == _lib.NFDPF_EINVAL
    assert b"null" in lib.nfdpf_last_error()
    rc = lib.nfdpf_soft_resample(None, None, None, None, 1, 10, 2, 0.5, 0, None, None, None, None)
    assert rc == _lib.NFDPF_EINVAL
    d = _lib.FilterDesc()
    d.B, d.N, d.T, d.t, d.hidden = 1, 1, 1, 0, 8
    assert lib.nfdpf_filter_step(ctypes.byref(d), None) == _lib.NFDPF_EINVAL
    assert b"N >= 2" in lib.nfdpf_last_error()
    assert lib.nfdpf_ot_workspace_bytes(64, 1000) > 64 * 1000 * 4 * 8


def test_ctypes_signatures_match_header_arity():
    """Every ctypes binding (nfdpf/_lib.py SIGNATURES) passes as many arguments as the header
    prototype declares -- a drift here would shift every later argument at the C ABI."""
    import re
    from nfdpf import _lib
    txt = re.sub(r"/\*.*?\*/", "", open(HEADER).read(), flags=re.S)
    protos = dict(re.findall(r"NFDPF_API\s+[\w\s\*]+?\b(nfdpf_\w+)\s*\(([^)]*)\)", txt))
    assert set(_lib.SIGNATURES) <= set(protos), sorted(set(_lib.SIGNATURES) - set(protos))
    for name, (_, argtypes) in _lib.SIGNATURES.items():
        params = protos[name].strip()
        n = 0 if params in ("", "void") else params.count(",") + 1
        assert len(argtypes) == n, f"{name}: ctypes passes {len(argtypes)} arguments, the header declares {n}"


def test_filter_desc_mirror_matches_library():
    """nfdpf._lib.FilterDesc mirrors nfdpf_filter_desc field by field; the library reports the
    struct size it was built with (load() refuses a mismatch -- a stale .so or binding)."""
    import ctypes
    from nfdpf import _lib
    assert int(_lib.load().nfdpf_filter_desc_size()) == ctypes.sizeof(_lib.FilterDesc)
