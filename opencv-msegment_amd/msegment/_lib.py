"""ctypes binding of libmsegment.so (the C ABI declared in include/msegment.h).

There is deliberately NO fallback: if the HIP library is missing or fails to load, every entry
point raises.  The CPU restatement under oracle/ is test infrastructure and is never imported
here.
"""
import ctypes
import hashlib
import os
import subprocess

_HERE = os.path.dirname(os.path.abspath(__file__))
# MSEGMENT_LIB overrides the in-tree library (A/B timing of alternative builds of the same ABI)
LIB_PATH = os.environ.get("MSEGMENT_LIB") or os.path.join(_HERE, "libmsegment.so")
CSRC = os.path.join(os.path.dirname(_HERE), "csrc")

MSG_OK = 0
MSG_EINVAL = -1
MSG_EHIP = -2
MSG_ENOMEM = -3
MSG_ETIMEOUT = -4
MSG_ESTATE = -5
MSG_ERANGE = -6

MSG_NC_GISTO_DIAP = 0x1
MSG_NC_MULTI_OTSU = 0x2
MSG_CREATE_HIGH_PRIORITY = 0x1
MSG_NC_MEDIAN_BLUR = 0x4
MSG_NC_BILATERAL = 0x8


def MSG_NC_MASK(k):
    return (int(k) & 0xff) << 8

# every symbol include/msegment.h declares (checked by tests/test_abi.py)
EXPORTS = (
    "msg_create", "msg_destroy", "msg_last_error", "msg_abi_version", "msg_build_id", "msg_get_stats",
    "msg_watershed", "msg_colorize", "msg_watershed_colorize", "msg_watershed_batch", "msg_watershed_colorize_batch",
    "msg_watershed_dev", "msg_colorize_dev", "msg_watershed_colorize_dev", "msg_edge_weights_dev",
    "msg_set_profiling", "msg_get_kernel_profile", "msg_set_diag", "msg_set_speculative",
    "msg_set_fast_commit",
    "msg_set_batch_inflight", "msg_set_batch_floods", "msg_set_batch_devices", "msg_set_resolve_grid", "msg_watershed_colorize_batch_dev",
    "msg_gray_hist_dev", "msg_nc_levels", "msg_nc_marker_lut", "msg_nc_markers_dev",
    "msg_nc_marker_stage_dev", "msg_nc_marker_stage",
    "msg_blur_mask_size", "msg_shape_markers_dev", "msg_shape_markers",
    "msg_color_markers_dev", "msg_color_markers",
)


class MsegError(RuntimeError):
    """Raised for a nonzero libmsegment return code (the CvException analogue)."""

    def __init__(self, code, msg):
        super().__init__("libmsegment error %d: %s" % (code, msg))
        self.code = code


class Stats(ctypes.Structure):
    _fields_ = [("batches", ctypes.c_int64), ("pops", ctypes.c_int64),
                ("host_syncs", ctypes.c_int64), ("rows", ctypes.c_int64), ("cols", ctypes.c_int64),
                ("items", ctypes.c_int64), ("pushes", ctypes.c_int64),
                ("diag", ctypes.c_int64 * 8),
                ("spec_generations", ctypes.c_int64), ("spec_rounds", ctypes.c_int64),
                ("spec_executions", ctypes.c_int64), ("spec_cascade_pops", ctypes.c_int64),
                ("spec_fallbacks", ctypes.c_int64), ("spec_replays", ctypes.c_int64),
                ("spec_cooldowns", ctypes.c_int64), ("spec_gen_pops", ctypes.c_int64),
                ("spec_gen_us", ctypes.c_int64),
                ("fast_pops", ctypes.c_int64), ("fast_pushes", ctypes.c_int64),
                ("scatter_pops", ctypes.c_int64), ("scatter_pushes", ctypes.c_int64),
                ("resolve_items", ctypes.c_int64), ("spec_exec_pops", ctypes.c_int64),
                ("spec_longest_pops", ctypes.c_int64), ("batch_mode", ctypes.c_int64),
                ("batch_probe", ctypes.c_int64)]


class KernelProfile(ctypes.Structure):
    _fields_ = [("name", ctypes.c_char * 32), ("launches", ctypes.c_int64), ("total_ms", ctypes.c_double)]


class BrightLevel(ctypes.Structure):
    """msg_bright_level = model/BrightLevel.java {start, end, count}."""

    _fields_ = [("start", ctypes.c_int32), ("end", ctypes.c_int32), ("count", ctypes.c_int32)]


NKERNELS = 24  # MSG_NKERNELS (include/msegment.h; tests/test_abi.py checks the two agree)


def build(arch="gfx950"):
    """Compile libmsegment.so in-tree with hipcc (no GPU needed)."""
    subprocess.check_call(["make", "-s", "-C", CSRC, "ARCH=%s" % arch])


def source_id(csrc=CSRC):
    """The id libmsegment.so carries (msg_build_id): SHA-256 prefix of csrc's sources (sorted by
    name) followed by include/msegment.h -- the same bytes the Makefile's BUILD_ID hashes."""
    names = sorted(f for f in os.listdir(csrc) if f.endswith((".hip", ".h", ".cpp")))
    paths = [os.path.join(csrc, f) for f in names]
    paths.append(os.path.join(os.path.dirname(os.path.dirname(csrc)), "include", "msegment.h"))
    h = hashlib.sha256()
    for p in paths:
        with open(p, "rb") as f:
            h.update(f.read())
    return h.hexdigest()[:16]


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(LIB_PATH):
        raise ImportError("libmsegment.so not built at %s (run __graft_entry__.build())" % LIB_PATH)
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7.  If it is
    # importable, load it first so libmsegment's DT_NEEDED binds to that same runtime (same
    # SONAME) and device pointers/streams from torch tensors are valid in both.  Loading ours
    # first would pull /opt/rocm's copy and torch would later fail with "No HIP GPUs".
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    L = ctypes.CDLL(LIB_PATH)
    L.msg_build_id.argtypes = []
    L.msg_build_id.restype = ctypes.c_char_p
    if not os.environ.get("MSEGMENT_LIB") and os.path.isdir(CSRC):
        # the in-tree library must be built from the sources next to it: a stale .so (shipped to a
        # box that did not rebuild) would silently run old kernels.  MSEGMENT_LIB (A/B builds of
        # other variants) is taken as given.
        built, want = L.msg_build_id().decode(), source_id()
        if built != want:
            raise ImportError("libmsegment.so is stale: built from sources %s, csrc/ is %s "
                              "(run __graft_entry__.build())" % (built, want))
    vp = ctypes.c_void_p
    sz = ctypes.c_size_t
    i = ctypes.c_int
    L.msg_create.argtypes = [ctypes.POINTER(vp), i, ctypes.c_uint]
    L.msg_create.restype = i
    L.msg_destroy.argtypes = [vp]
    L.msg_destroy.restype = None
    L.msg_last_error.argtypes = [vp]
    L.msg_last_error.restype = ctypes.c_char_p
    L.msg_abi_version.argtypes = []
    L.msg_abi_version.restype = i
    L.msg_get_stats.argtypes = [vp, ctypes.POINTER(Stats)]
    L.msg_get_stats.restype = i
    L.msg_watershed.argtypes = [vp, vp, sz, vp, sz, i, i]
    L.msg_watershed.restype = i
    L.msg_colorize.argtypes = [vp, vp, sz, i, i, i, vp, vp, sz]
    L.msg_colorize.restype = i
    L.msg_watershed_colorize.argtypes = [vp, vp, sz, vp, sz, i, i, i, vp, vp, sz, vp, sz]
    L.msg_watershed_colorize.restype = i
    L.msg_watershed_batch.argtypes = [vp, i, vp, vp, vp, vp, vp, vp]
    L.msg_watershed_batch.restype = i
    L.msg_watershed_colorize_batch.argtypes = [vp, i, vp, vp, vp, vp, vp, vp, i, vp, vp, vp]
    L.msg_watershed_colorize_batch.restype = i
    L.msg_watershed_dev.argtypes = [vp, vp, vp, vp, i, i, vp]
    L.msg_watershed_dev.restype = i
    L.msg_colorize_dev.argtypes = [vp, vp, i, i, i, vp, vp, vp, vp]
    L.msg_colorize_dev.restype = i
    L.msg_watershed_colorize_dev.argtypes = [vp, vp, vp, vp, i, i, i, vp, vp, vp, vp]
    L.msg_watershed_colorize_dev.restype = i
    L.msg_edge_weights_dev.argtypes = [vp, vp, vp, vp, i, i, vp]
    L.msg_edge_weights_dev.restype = i
    L.msg_set_profiling.argtypes = [vp, i]
    L.msg_set_profiling.restype = i
    L.msg_set_diag.argtypes = [vp, i]
    L.msg_set_diag.restype = i
    L.msg_set_speculative.argtypes = [vp, i]
    L.msg_set_speculative.restype = i
    L.msg_set_fast_commit.argtypes = [vp, i]
    L.msg_set_fast_commit.restype = i
    L.msg_get_kernel_profile.argtypes = [vp, ctypes.POINTER(KernelProfile), i, i]
    L.msg_get_kernel_profile.restype = i
    L.msg_set_batch_inflight.argtypes = [vp, i]
    L.msg_set_batch_inflight.restype = i
    if hasattr(L, "msg_set_batch_floods"):  # (MSEGMENT_LIB A/B builds of earlier rounds lack it)
        L.msg_set_batch_floods.argtypes = [vp, i]
        L.msg_set_batch_floods.restype = i
    if hasattr(L, "msg_set_batch_devices"):  # (ABI 7)
        L.msg_set_batch_devices.argtypes = [vp, i, vp]
        L.msg_set_batch_devices.restype = i
    L.msg_set_resolve_grid.argtypes = [vp, i]
    L.msg_set_resolve_grid.restype = i
    L.msg_watershed_colorize_batch_dev.argtypes = [vp, i, vp, vp, vp, vp, vp, i, vp, vp, vp]
    L.msg_watershed_colorize_batch_dev.restype = i
    L.msg_gray_hist_dev.argtypes = [vp, vp, i, i, vp, vp, vp]
    L.msg_gray_hist_dev.restype = i
    L.msg_nc_levels.argtypes = [vp, i, i, i, ctypes.c_uint, ctypes.POINTER(BrightLevel), i,
                                ctypes.POINTER(i)]
    L.msg_nc_levels.restype = i
    L.msg_nc_marker_lut.argtypes = [ctypes.POINTER(BrightLevel), i, ctypes.c_uint, vp]
    L.msg_nc_marker_lut.restype = i
    L.msg_nc_markers_dev.argtypes = [vp, vp, i, i, vp, vp, vp]
    L.msg_nc_markers_dev.restype = i
    L.msg_nc_marker_stage_dev.argtypes = [vp, vp, i, i, i, ctypes.c_uint, vp, vp,
                                          ctypes.POINTER(BrightLevel), i, ctypes.POINTER(i), vp]
    L.msg_nc_marker_stage_dev.restype = i
    L.msg_nc_marker_stage.argtypes = [vp, vp, sz, i, i, i, ctypes.c_uint, vp, sz,
                                      ctypes.POINTER(BrightLevel), i, ctypes.POINTER(i)]
    L.msg_nc_marker_stage.restype = i
    L.msg_blur_mask_size.argtypes = [i, i]
    L.msg_blur_mask_size.restype = i
    L.msg_shape_markers_dev.argtypes = [vp, vp, i, i, i, vp, ctypes.POINTER(i), ctypes.POINTER(i),
                                        vp, vp, vp, vp]
    L.msg_shape_markers_dev.restype = i
    L.msg_shape_markers.argtypes = [vp, vp, sz, i, i, i, vp, sz, ctypes.POINTER(i), ctypes.POINTER(i)]
    L.msg_shape_markers.restype = i
    L.msg_color_markers_dev.argtypes = [vp, vp, i, i, vp, vp, ctypes.POINTER(i), vp]
    L.msg_color_markers_dev.restype = i
    L.msg_color_markers.argtypes = [vp, vp, sz, i, i, vp, sz, vp, sz, ctypes.POINTER(i)]
    L.msg_color_markers.restype = i
    _lib = L
    return L
