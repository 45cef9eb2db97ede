"""CPU: the C-ABI library loads and exports every symbol include/msegment.h declares.
No compute calls (there is no GPU in the build container)."""
import ctypes
import os
import re

from msegment import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "msegment.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(msg_[a-z_0-9]+)\s*\(", hdr)))


def test_library_exports_header_symbols():
    L = ctypes.CDLL(_lib.LIB_PATH)
    syms = declared_symbols()
    assert len(syms) >= 12
    for s in syms:
        assert hasattr(L, s), s
    assert set(syms) == set(_lib.EXPORTS)


def test_abi_version_and_binding_load():
    L = _lib.load()
    assert L.msg_abi_version() == 7


def test_build_id_matches_sources():
    """libmsegment.so is built from the csrc/ next to it (msg_build_id = the Makefile's BUILD_ID);
    _lib.load() refuses a stale library."""
    L = _lib.load()
    assert L.msg_build_id().decode() == _lib.source_id()


def test_stats_struct_matches_header():
    """The ctypes Stats mirror has exactly the header's msg_stats fields (all int64): a smaller
    caller struct would be overrun by msg_get_stats."""
    hdr = open(os.path.join(ROOT, "include", "msegment.h")).read()
    body = re.search(r"typedef struct msg_stats \{(.*?)\} msg_stats;", hdr, flags=re.S).group(1)
    body = re.sub(r"/\*.*?\*/", "", body, flags=re.S)
    n = 0
    for decl in re.findall(r"int64_t\s+([^;]+);", body):
        for name in decl.split(","):
            m = re.match(r"\s*(\w+)\s*(?:\[(\d+)\])?", name)
            n += int(m.group(2)) if m.group(2) else 1
    assert ctypes.sizeof(_lib.Stats) == 8 * n


def test_library_is_gfx950_code_object():
    data = open(_lib.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_null_context_is_rejected_without_gpu():
    L = _lib.load()
    assert L.msg_watershed(None, None, 0, None, 0, 4, 4) == _lib.MSG_EINVAL
    assert L.msg_create(None, 0, 0) == _lib.MSG_EINVAL


def test_python_constants_match_header():
    """The ctypes mirror's constants (msegment/_lib.py) equal include/msegment.h's #defines: a
    stale NKERNELS would cut the kernel profile short, a stale option bit would select the wrong
    pre-filter."""
    import re

    from msegment import _lib

    hdr = open(os.path.join(os.path.dirname(__file__), "..", "include", "msegment.h")).read()
    defs = dict(re.findall(r"#define (MSG_\w+)\s+\(?(-?(?:0x)?[0-9a-fA-F]+)u?\)?", hdr))
    assert int(defs["MSG_NKERNELS"], 0) == _lib.NKERNELS
    for name in ("MSG_OK", "MSG_EINVAL", "MSG_EHIP", "MSG_ENOMEM", "MSG_ETIMEOUT", "MSG_ESTATE", "MSG_ERANGE",
                 "MSG_NC_GISTO_DIAP", "MSG_NC_MULTI_OTSU", "MSG_NC_MEDIAN_BLUR", "MSG_NC_BILATERAL",
                 "MSG_CREATE_HIGH_PRIORITY"):
        assert int(defs[name], 0) == getattr(_lib, name), name
