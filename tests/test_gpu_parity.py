"""GPU parity: libmsegment (HIP, gfx950) vs the CPU oracle, bit-exact on int32 labels and on
the colourised / gray bytes.  Everything goes through the C ABI (include/msegment.h)."""
import hashlib
import json
import os

import numpy as np
import pytest

from oracle import ws_oracle
from msegment import synth
from msegment.jrandom import generate_bgr_palette

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def gpu_ws(seg, img, m):
    out = np.array(m, dtype=np.int32, copy=True)
    seg.watershed(img, out)
    return out


def test_kats(seg):
    img = np.zeros((5, 5, 3), np.uint8)
    m = np.zeros((5, 5), np.int32)
    m[1, 1], m[3, 3] = 1, 2
    want = np.array([[-1, -1, -1, -1, -1], [-1, 1, 1, -1, -1], [-1, 1, -1, 2, -1],
                     [-1, -1, 2, 2, -1], [-1, -1, -1, -1, -1]], np.int32)
    assert np.array_equal(gpu_ws(seg, img, m), want)
    m = np.zeros((3, 3), np.int32)
    m[0, 0] = 5
    out = gpu_ws(seg, np.zeros((3, 3, 3), np.uint8), m)
    assert out[1, 1] == 0 and (out != 0).sum() == 8
    m = np.zeros((3, 3), np.int32)
    m[1, 1] = -7
    assert gpu_ws(seg, np.zeros((3, 3, 3), np.uint8), m)[1, 1] == 0
    for shape in [(1, 1), (1, 7), (2, 2), (7, 1), (2, 9), (9, 2)]:
        assert (gpu_ws(seg, np.zeros(shape + (3,), np.uint8), np.ones(shape, np.int32)) == -1).all()


def test_empty_frames(seg):
    for shape in [(0, 0), (0, 5), (5, 0)]:
        m = np.zeros(shape, np.int32)
        seg.watershed(np.zeros(shape + (3,), np.uint8), m)


def test_golden_small_cases(seg):
    z = np.load(os.path.join(GOLD, "small_cases.npz"))
    for n in list(z["__names"]):
        img, m, d = z[n + "__img"], z[n + "__markers"], int(z[n + "__depth"])
        work = m.copy()
        dst, gray = seg.watershed_colorize(img, work, d, z[n + "__palette"], gray=True)
        assert np.array_equal(work, z[n + "__labels"]), n
        assert np.array_equal(dst, z[n + "__color"]), n
        assert np.array_equal(gray, z[n + "__gray"]), n
        assert np.array_equal(seg.colorize(work, d, None), z[n + "__white"]), n


def test_random_small_vs_oracle(seg):
    rng = np.random.default_rng(7)
    for t in range(150):
        H, W = (int(v) for v in rng.integers(1, 48, 2))
        img = rng.integers(0, 256, (H, W, 3), dtype=np.uint8)
        q = t % 4
        if q == 0:
            img = (img // 128 * 128).astype(np.uint8)
        elif q == 1:
            img = (img // 32).astype(np.uint8)
        elif q == 2:
            img[:] = img[0, 0]
        m = np.zeros((H, W), np.int32)
        for _ in range(int(rng.integers(0, 16))):
            m[rng.integers(0, H), rng.integers(0, W)] = rng.integers(-4, 7)
        assert np.array_equal(gpu_ws(seg, img, m), ws_oracle.watershed(img, m)), (t, H, W)


def test_dense_and_adjacent_seeds(seg):
    rng = np.random.default_rng(11)
    for t in range(20):
        H, W = 37, 53
        img = (rng.integers(0, 256, (H, W, 3), dtype=np.uint8) // (64 if t % 2 else 1)).astype(np.uint8)
        m = rng.integers(-2, 9, (H, W)).astype(np.int32) * (rng.random((H, W)) < 0.3)
        assert np.array_equal(gpu_ws(seg, img, m.astype(np.int32)), ws_oracle.watershed(img, m)), t


def test_strided_views_in_place(seg):
    img, m, d = synth.frame("mosaic_noise", 70, 90, 5)
    big_img = np.zeros((70, 100, 3), np.uint8)
    big_img[:, :90] = img
    big_m = np.full((70, 97), 12345, np.int32)
    big_m[:, :90] = m
    view = big_m[:, :90]
    seg.watershed(big_img[:, :90], view)
    assert np.array_equal(view, ws_oracle.watershed(img, m))
    assert (big_m[:, 90:] == 12345).all()


@pytest.mark.parametrize("kind,H,W,seed", [("mosaic", 256, 256, 0), ("mosaic_noise", 256, 256, 3),
                                           ("random", 192, 160, 4), ("mosaic_noise", 333, 517, 8)])
def test_synthetic_vs_oracle(seg, kind, H, W, seed):
    img, m, d = synth.frame(kind, H, W, seed)
    assert np.array_equal(gpu_ws(seg, img, m), ws_oracle.watershed(img, m))


def test_config2_1024_mosaic_digest(seg):
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_1024x1024_s1"]
    img, m, d = synth.frame("mosaic", 1024, 1024, 1)
    out = gpu_ws(seg, img, m)
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]


def test_config3_4096_mosaic_digest_and_properties(seg):
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_4096x4096_s2"]
    img, m, d = synth.frame("mosaic", 4096, 4096, 2)
    out = gpu_ws(seg, img, m)
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]
    check_properties(m, out)


@pytest.mark.parametrize("kind", ["mosaic_noise", "random"])
def test_config3_4096_stress_digest_and_properties(seg, kind):
    """BASELINE config 3's stress variants (mosaic+noise, uniform-random; 4096^2, seed 2): the
    interrupt-dense regime at full size, against the oracle's digest, plus the invariants."""
    key = "%s_4096x4096_s2" % kind
    dg = json.load(open(os.path.join(GOLD, "digests.json")))[key]
    img, m, d = synth.frame(kind, 4096, 4096, 2)
    out = gpu_ws(seg, img, m)
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]
    assert int((out == -1).sum()) == dg["wshed_pixels"]
    check_properties(m, out)


def test_config4_16384_mosaic_digest_single_gpu(seg):
    """BASELINE config 4's frame (16384^2, SURVEY.md seed 3) on ONE GPU: the 2^28-pixel frame's
    ~12 GB workspace fits one MI355X (why it is not tile-sharded)."""
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_16384x16384_s3"]
    img, m, d = synth.frame("mosaic", 16384, 16384, 3)
    out = gpu_ws(seg, img, m)
    del img
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]
    assert int((out == -1).sum()) == dg["wshed_pixels"]


def test_frame_above_2_28_pixels_digest(seg):
    """16387 x 32749 = 537 M pixels (2x config 4, ragged 4x4 tiles in both directions): above
    round 1's 2^28-pixel limit and just below the flood's 32-bit index limit (4N + 16 queue slots,
    check_size), against the oracle's digest (tests/golden/make_golden.py)."""
    import torch

    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_16387x32749_s11"]
    img, m, d = synth.frame("mosaic", 16387, 32749, 11)
    assert hashlib.sha256(m.tobytes()).hexdigest() == dg["markers_sha256"]
    dev = torch.device("cuda", seg.device)
    t_img = torch.from_numpy(img).to(dev)
    del img
    t_m = torch.from_numpy(m).to(dev)
    del m
    seg.watershed_dev(t_img, t_m, t_m)
    torch.cuda.synchronize(dev)
    del t_img
    out = t_m.cpu().numpy()
    del t_m
    torch.cuda.empty_cache()
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]
    assert int((out == -1).sum()) == dg["wshed_pixels"]


def test_large_ragged_mosaic_digest(seg):
    """3001 x 5003: ragged 4x4 tiles in both directions (3001 % 4 == 1, 5003 % 4 == 3) at 15 M
    pixels, against the oracle's digest, plus the invariants."""
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_3001x5003_s7"]
    img, m, d = synth.frame("mosaic", 3001, 5003, 7)
    out = gpu_ws(seg, img, m)
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]
    check_properties(m, out)


def test_config5_frames_batch_vs_digest(seg):
    """BASELINE config 5's frames (4096^2, SURVEY.md seeds 100 + k) through the device batch entry
    point, 4 floods in flight: all 8 frames of the batch bench.py times, each against the oracle's
    digest of that frame (tests/golden/digests.json)."""
    import torch

    dev = torch.device("cuda", seg.device)
    dgs = json.load(open(os.path.join(GOLD, "digests.json")))
    fr = [synth.frame("mosaic", 4096, 4096, 100 + k) for k in range(8)]
    depth = max(f[2] for f in fr)
    imgs = [torch.from_numpy(f[0]).to(dev) for f in fr]
    mks = [torch.from_numpy(f[1]).to(dev) for f in fr]
    labs = [torch.empty_like(x) for x in mks]
    dsts = [torch.empty((4096, 4096, 3), dtype=torch.uint8, device=dev) for _ in fr]
    seg.set_batch_inflight(4)
    seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
    torch.cuda.synchronize()
    for k in range(8):
        got = labs[k].cpu().numpy()
        assert hashlib.sha256(got.tobytes()).hexdigest() == dgs["mosaic_4096x4096_s%d" % (100 + k)]["labels_sha256"], k


def test_config5_multi_device_batch_vs_digest(seg):
    """Config 5 through the multi-device C-ABI entry (msg_set_batch_devices) as the JVM reaches it:
    the device list [0, 0] (two sub-contexts on the one GPU of the box, 4 frames each, each with its
    own floods in flight), host buffers, colorByIndexes; all 8 frames against the oracle digests,
    the colours against the oracle's colouring of the digest-checked labels; then a bad list and
    the reset to the context's own device."""
    import msegment

    dgs = json.load(open(os.path.join(GOLD, "digests.json")))
    fr = [synth.frame("mosaic", 4096, 4096, 100 + k) for k in range(8)]
    depth = max(f[2] for f in fr)
    work = [(f[0], f[1].copy()) for f in fr]
    seg.set_batch_devices([0, 0])
    try:
        dsts = seg.watershed_batch(work, depth=depth)
        st = seg.stats()
        with pytest.raises(msegment.MsegError):
            seg.set_batch_devices([0, 4096])
    finally:
        seg.set_batch_devices([])
    assert st["rows"] == 4096 and st["pops"] > 8 * 4000 * 4000  # the sums over both sub-contexts
    for k, (_, lab) in enumerate(work):
        assert hashlib.sha256(lab.tobytes()).hexdigest() == dgs["mosaic_4096x4096_s%d" % (100 + k)]["labels_sha256"], k
    for k in (0, 7):  # first frame of each block
        assert np.array_equal(dsts[k], ws_oracle.colorize(work[k][1], depth, None)), k
    # back on the context's own device
    img, m, _ = synth.frame("mosaic_noise", 96, 80, 5)
    w2 = [(img, m.copy())]
    seg.watershed_batch(w2)
    assert np.array_equal(w2[0][1], ws_oracle.watershed(img, m))


def check_properties(m, out):
    """Size-independent watershed invariants."""
    H, W = m.shape
    assert (out[0] == -1).all() and (out[-1] == -1).all() and (out[:, 0] == -1).all() and (out[:, -1] == -1).all()
    seeds = set(np.unique(m[1:-1, 1:-1][m[1:-1, 1:-1] > 0]).tolist())
    labs = set(np.unique(out[out > 0]).tolist())
    assert labs <= seeds
    inner = m[1:-1, 1:-1] > 0
    assert np.array_equal(out[1:-1, 1:-1][inner], m[1:-1, 1:-1][inner])  # seeds never change
    # two 4-adjacent pixels with different positive labels are both input seeds
    for a, b, sa, sb in [(out[:, :-1], out[:, 1:], m[:, :-1], m[:, 1:]), (out[:-1], out[1:], m[:-1], m[1:])]:
        bad = (a > 0) & (b > 0) & (a != b)
        assert ((sa[bad] > 0) & (sb[bad] > 0)).all()
    assert not (out == -2).any()


def test_noise_1024_vs_oracle(seg):
    img, m, d = synth.frame("mosaic_noise", 1024, 1024, 1)
    out = gpu_ws(seg, img, m)
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_noise_1024x1024_s1"]
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]


def test_repeated_calls_same_context(seg):
    img, m, d = synth.frame("mosaic_noise", 128, 128, 2)
    want = ws_oracle.watershed(img, m)
    for _ in range(5):
        assert np.array_equal(gpu_ws(seg, img, m), want)
    # a bigger frame then a smaller one (workspace reuse)
    img2, m2, _ = synth.frame("mosaic", 600, 400, 9)
    assert np.array_equal(gpu_ws(seg, img2, m2), ws_oracle.watershed(img2, m2))
    assert np.array_equal(gpu_ws(seg, img, m), want)


def test_batch_api(seg):
    frames = [synth.frame("mosaic_noise", 64 + 8 * k, 80, 100 + k)[:2] for k in range(4)]
    work = [(img, m.copy()) for img, m in frames]
    seg.watershed_batch(work)
    for (img, m), (_, out) in zip(frames, work):
        assert np.array_equal(out, ws_oracle.watershed(img, m))


@pytest.mark.parametrize("inflight", [1, 3, 8])
def test_batch_api_inflight(seg, inflight):
    """Several floods in flight (internal sub-contexts, one host thread each), frames of mixed
    sizes and kinds; every frame bit-exact and written back to its own markers."""
    frames = [synth.frame(("mosaic", "mosaic_noise")[k % 2], 60 + 17 * k, 90 + 5 * k, 200 + k)[:2]
              for k in range(7)]
    work = [(img, m.copy()) for img, m in frames]
    seg.set_batch_inflight(inflight)
    try:
        seg.watershed_batch(work)
    finally:
        seg.set_batch_inflight(4)
    for (img, m), (_, out) in zip(frames, work):
        assert np.array_equal(out, ws_oracle.watershed(img, m))


def test_batch_dev_inflight(seg):
    import torch

    dev = torch.device("cuda", seg.device)
    frames = [synth.frame(("mosaic", "mosaic_noise", "random")[k % 3], 100 + 31 * k, 140 - 9 * k, 300 + k)
              for k in range(6)]
    depth = max(f[2] for f in frames)
    pal = generate_bgr_palette(depth, 11)
    t_pal = torch.from_numpy(pal).to(dev)
    bgrs = [torch.from_numpy(f[0]).to(dev) for f in frames]
    mks = [torch.from_numpy(f[1]).to(dev) for f in frames]
    labs = [torch.empty_like(m) for m in mks]
    dsts = [torch.empty((m.shape[0], m.shape[1], 3), dtype=torch.uint8, device=dev) for m in mks]
    seg.set_batch_inflight(3)
    try:
        seg.watershed_colorize_batch_dev(bgrs, mks, labs, depth, t_pal, dsts)
    finally:
        seg.set_batch_inflight(4)
    for f, lab, dst in zip(frames, labs, dsts):
        want = ws_oracle.watershed(f[0], f[1])
        assert np.array_equal(lab.cpu().numpy(), want)
        assert np.array_equal(dst.cpu().numpy(), ws_oracle.colorize(want, depth, pal))


def test_colorize_palette_sizes(seg):
    rng = np.random.default_rng(3)
    for depth in [0, 1, 7, 5000, 20000, 70000]:
        lab = rng.integers(-2, depth + 3, (61, 77)).astype(np.int32)
        pal = generate_bgr_palette(depth, depth + 1)
        assert np.array_equal(seg.colorize(lab, depth, pal), ws_oracle.colorize(lab, depth, pal)), depth
        assert np.array_equal(seg.colorize(lab, depth, None), ws_oracle.colorize(lab, depth, None)), depth


def test_invalid_arguments(seg):
    import msegment

    with pytest.raises(msegment.MsegError):
        seg.watershed(np.zeros((4, 4, 3), np.uint8), np.zeros((4, 5), np.int32))
    with pytest.raises(msegment.MsegError):
        seg.watershed(np.zeros((4, 4), np.uint8), np.zeros((4, 4), np.int32))
    with pytest.raises(msegment.MsegError):
        seg.watershed(np.zeros((4, 4, 3), np.uint8), np.zeros((4, 4), np.float32))


def test_device_api_torch(seg):
    import torch

    img, m, d = synth.frame("mosaic_noise", 300, 260, 6)
    pal = generate_bgr_palette(d, 5)
    dev = torch.device("cuda", seg.device)
    t_img = torch.from_numpy(img).to(dev)
    t_m = torch.from_numpy(m).to(dev)
    t_lab = torch.empty_like(t_m)
    t_pal = torch.from_numpy(pal).to(dev)
    t_dst = torch.empty((300, 260, 3), dtype=torch.uint8, device=dev)
    t_gray = torch.empty((300, 260), dtype=torch.uint8, device=dev)
    seg.watershed_colorize_dev(t_img, t_m, t_lab, d, t_pal, t_dst, t_gray)
    torch.cuda.synchronize()
    want = ws_oracle.watershed(img, m)
    assert np.array_equal(t_lab.cpu().numpy(), want)
    assert np.array_equal(t_m.cpu().numpy(), m)  # out-of-place: input untouched
    col = ws_oracle.colorize(want, d, pal)
    assert np.array_equal(t_dst.cpu().numpy(), col)
    assert np.array_equal(t_gray.cpu().numpy(), ws_oracle.bgr2gray(col))


@pytest.mark.parametrize("shape", [(123, 77), (64, 256), (17, 16), (1, 32), (33, 48), (2, 15), (4101, 8192)])
def test_edge_weights_dev(seg, shape):
    """Both stencil kernels: width % 16 == 0 takes the 16-pixel vector path (2 rows per thread up to
    2 x 4096^2 pixels, 4 above: the 4101 x 8192 case, with a ragged last strip)."""
    import torch

    H, W = shape
    img = synth.random_image(H, W, 1 + H)
    dev = torch.device("cuda", seg.device)
    t = torch.from_numpy(img).to(dev)
    wr = torch.empty((H, W), dtype=torch.uint8, device=dev)
    wd = torch.empty_like(wr)
    seg.edge_weights_dev(t, wr, wd)
    torch.cuda.synchronize()
    x = img.astype(np.int32)
    er = np.zeros((H, W), np.uint8)
    ed = np.zeros((H, W), np.uint8)
    er[:, :-1] = np.abs(x[:, 1:] - x[:, :-1]).max(axis=2)
    ed[:-1] = np.abs(x[1:] - x[:-1]).max(axis=2)
    assert np.array_equal(wr.cpu().numpy(), er) and np.array_equal(wd.cpu().numpy(), ed)


def test_picture_service_mirror(seg):
    import msegment

    img, m, d = synth.frame("mosaic", 128, 96, 12)
    ps = msegment.PictureService(segmenter=seg, seed=99)
    work = m.copy()
    dst = ps.watershed(img, work, d, True)
    want = ws_oracle.watershed(img, m)
    assert np.array_equal(work, want)
    assert np.array_equal(dst, ws_oracle.colorize(want, d, generate_bgr_palette(d, 99)))
    work = m.copy()
    assert np.array_equal(ps.watershed(img, work, d, False), ws_oracle.colorize(want, d, None))


def test_batch_inflight_more_hw_queues():
    """Regression: with more hardware queues than the default 4, 8 concurrent 4096^2 floods used
    to time out in k_resolve's cross-rank waits (their grids were not all co-resident).  k_resolve
    now deals rank chunks in dispatch order, and every flood keeps the full grid (no budget
    split).  Runs in a child process (the queue count is fixed when HIP initialises); labels must
    equal the same frames flooded one at a time."""
    import subprocess
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, GPU_MAX_HW_QUEUES="16")
    r = subprocess.run([sys.executable, os.path.join(root, "scripts", "stress_inflight_dev.py"),
                        "6", "8", "8", "4096"], env=env, capture_output=True, text=True, timeout=110)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    assert "0 error steps, 0 bad frames" in r.stdout


def test_c_abi_error_paths(seg):
    """The C ABI's CV_Assert-like checks (include/msegment.h): each bad call returns MSG_EINVAL
    with a message and leaves the context usable."""
    import ctypes

    from msegment import _lib

    L, h = seg._L, seg._h
    img = np.zeros((8, 8, 3), np.uint8)
    mk = np.zeros((8, 8), np.int32)
    mk[4, 4] = 1
    ip = img.ctypes.data_as(ctypes.c_void_p)
    mp = mk.ctypes.data_as(ctypes.c_void_p)
    bad = [
        lambda: L.msg_watershed(h, ip, 24, mp, 32, -1, 8),          # negative rows
        lambda: L.msg_watershed(h, ip, 24, mp, 32, 1 << 15, 1 << 14),  # 2^29 pixels: 4N slots overflow
        lambda: L.msg_watershed(h, ip, 24, mp, 32, 1, (1 << 29) - 1024),  # 1-row frame: 4x4 tile padding overflows
        lambda: L.msg_watershed(h, None, 24, mp, 32, 8, 8),         # null image
        lambda: L.msg_watershed(h, ip, 23, mp, 32, 8, 8),           # bgr stride < 3 cols
        lambda: L.msg_watershed(h, ip, 24, mp, 30, 8, 8),           # marker stride not 4-aligned
        lambda: L.msg_watershed_colorize(h, ip, 24, mp, 32, 8, 8, -1, None,
                                         img.ctypes.data_as(ctypes.c_void_p), 24, None, 0),  # depth < 0
        lambda: L.msg_set_batch_inflight(h, 0),
    ]
    for k, call in enumerate(bad):
        assert call() == _lib.MSG_EINVAL, k
        assert L.msg_last_error(h), k
        if k in (1, 2):
            assert b"32-bit indices" in L.msg_last_error(h), k
    out = mk.copy()
    assert L.msg_watershed(h, ip, 24, out.ctypes.data_as(ctypes.c_void_p), 32, 8, 8) == 0
    assert np.array_equal(out, ws_oracle.watershed(img, mk))
    # empty frames are a no-op, not an error
    assert L.msg_watershed(h, ip, 24, mp, 32, 0, 8) == 0


@pytest.mark.parametrize("blocks", [1, 7, 16 * 256 * 4])
def test_resolve_grid_any_size(seg, blocks):
    """k_resolve's progress does not depend on co-residency: one block, a few, and a grid 16x
    larger than the device can hold all give the oracle's labels without MSG_ETIMEOUT."""
    img, m, d = synth.frame("mosaic", 1024, 1024, 1)
    dg = json.load(open(os.path.join(GOLD, "digests.json")))["mosaic_1024x1024_s1"]
    seg.set_resolve_grid(blocks)
    try:
        out = gpu_ws(seg, img, m)
    finally:
        seg.set_resolve_grid(0)
    assert hashlib.sha256(out.tobytes()).hexdigest() == dg["labels_sha256"]


@pytest.mark.parametrize("kind,S", [("mosaic", 1024), ("mosaic_noise", 300), ("random", 256)])
def test_resolve_give_up_and_rerun(seg, kind, S):
    """Fault injection (msg_set_diag 2): k_resolve's odd blocks give up their first chunk of every
    batch, so waiters on them give up too after their long-wait check, and k_scan re-runs the
    batch until every chunk has completed.  Labels must still be the oracle's."""
    img, m, d = synth.frame(kind, S, S, 5)
    seg.set_diag(2)
    try:
        out = gpu_ws(seg, img, m)
    finally:
        seg.set_diag(False)
    assert np.array_equal(out, ws_oracle.watershed(img, m))


@pytest.mark.parametrize("blocks", [4, 16])
def test_rerun_skips_with_many_chunks_per_block(seg, blocks):
    """Re-runs on a small k_resolve grid: every block walks many chunks, alternating completed
    (skipped) and re-run ones.  Regression: the skip flag was one shared word, so a wave that
    lagged behind a skipped chunk could read the next chunk's flag and redo a completed chunk out
    of step with its block (wrong bucket histograms, pixels queued twice; found as rare label
    differences with 8 concurrent floods).  Labels must be the oracle's."""
    img, m, d = synth.frame("mosaic", 1024, 1024, 9)
    seg.set_diag(2)
    seg.set_resolve_grid(blocks)
    try:
        out = gpu_ws(seg, img, m)
    finally:
        seg.set_diag(False)
        seg.set_resolve_grid(0)
    assert np.array_equal(out, ws_oracle.watershed(img, m))


def test_two_contexts_two_threads():
    """Two Segmenters flooding at the same time from two host threads (the one-context-per-thread
    model of include/msegment.h), each with the full k_resolve grid: both bit-exact."""
    import threading

    import msegment

    fr = [synth.frame("mosaic", 2048, 2048, 40 + k) for k in range(2)]
    want = [ws_oracle.watershed(img, m) for img, m, _ in fr]
    got = [None, None]
    errs = []

    def run(k):
        try:
            with msegment.Segmenter(0) as s:
                for _ in range(3):
                    got[k] = gpu_ws(s, fr[k][0], fr[k][1])
                    if not np.array_equal(got[k], want[k]):
                        break
        except Exception as e:  # noqa: BLE001
            errs.append(e)

    th = [threading.Thread(target=run, args=(k,)) for k in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join(timeout=100)
    assert not errs, errs
    for k in range(2):
        assert np.array_equal(got[k], want[k]), k


def test_default_stream_ordering_without_device_sync(seg):
    """Device calls on torch's default (legacy null) stream: the library orders its own stream
    after the null stream's queued work and the null stream after its own, so a chain of
    stream-ordered torch ops and library calls needs no device-wide synchronize.  The inputs are
    produced by a long torch kernel chain right before the call; the outputs are consumed by
    torch ops right after it."""
    import torch

    dev = torch.device("cuda", seg.device)
    img, m, d = synth.frame("mosaic_noise", 512, 640, 21)
    want = ws_oracle.watershed(img, m)
    big = torch.randn(3072, 3072, device=dev)
    for _ in range(3):
        t_img = torch.from_numpy(img).to(dev)
        t_m0 = torch.from_numpy(m).to(dev)
        x = big
        for _ in range(4):
            x = x @ big  # keep the null stream busy
        t_m = t_m0 + (x[0, 0] * 0).to(torch.int32)  # markers written by the last queued kernel
        t_lab = torch.empty_like(t_m)
        seg.watershed_dev(t_img, t_m, t_lab)
        dst = torch.empty((512, 640, 3), dtype=torch.uint8, device=dev)
        seg.colorize_dev(t_lab, d, None, dst)
        lab_copy = t_lab.clone()
        dst_copy = dst.clone()
        assert np.array_equal(lab_copy.cpu().numpy(), want)
        assert np.array_equal(dst_copy.cpu().numpy(), ws_oracle.colorize(want, d, None))


@pytest.mark.parametrize("W", [256, 259])
def test_prep_paths_on_misaligned_device_buffers(seg, W):
    """k_prep4 (quad loads: width divisible by 4, 4-B aligned BGR, 16-B aligned markers) and the
    tile-row k_prep (every other case) give the same flood: the same frame through aligned
    tensors and through tensors offset by one element (which forces k_prep) -- and the oracle."""
    import torch

    img, m, _ = synth.frame("mosaic_noise", 192, W, 21)
    want = ws_oracle.watershed(img, m)
    dev = torch.device("cuda", 0)
    outs = []
    for off in (0, 1):
        bimg = torch.zeros(img.size + 3 * off, dtype=torch.uint8, device=dev)
        bmk = torch.zeros(m.size + off, dtype=torch.int32, device=dev)
        timg = bimg[3 * off:].view(img.shape)
        tmk = bmk[off:].view(m.shape)
        timg.copy_(torch.from_numpy(img))
        tmk.copy_(torch.from_numpy(m))
        lab = torch.empty_like(tmk)
        seg.watershed_dev(timg, tmk, lab)
        torch.cuda.synchronize()
        outs.append(lab.cpu().numpy())
    assert np.array_equal(outs[0], want) and np.array_equal(outs[1], want)


@pytest.mark.parametrize("kind,S,seed", [("mosaic", 2048, 5), ("mosaic", 1024, 1), ("mosaic_noise", 512, 9)])
def test_fast_commit_matches_three_launch_iterations(seg, kind, S, seed):
    """k_commit_fast (two-launch iterations for batches of 4 K..256 K items) against the three-launch
    iterations and the oracle; the fast path must actually have run on the mosaic frames."""
    img, m, _ = synth.frame(kind, S, S, seed)
    want = ws_oracle.watershed(img, m)
    seg.set_profiling(True)
    try:
        seg.kernel_profile(reset=True)
        fast = gpu_ws(seg, img, m)
        prof = seg.kernel_profile(reset=True)
        seg.set_fast_commit(False)
        slow = gpu_ws(seg, img, m)
        prof_off = seg.kernel_profile(reset=True)
    finally:
        seg.set_fast_commit(True)
        seg.set_profiling(False)
    assert np.array_equal(fast, want) and np.array_equal(slow, want)
    assert prof_off.get("k_commit_fast", (0, 0))[0] == 0
    if kind == "mosaic":
        assert prof["k_commit_fast"][0] > 0


def test_fast_commit_with_give_ups(seg):
    """Injected k_resolve give-ups (msg_set_diag 2): k_commit_fast must schedule the re-run instead
    of committing; then the same context without injection."""
    img, m, _ = synth.frame("mosaic", 1024, 1024, 3)
    want = ws_oracle.watershed(img, m)
    seg.set_diag(2)
    try:
        assert np.array_equal(gpu_ws(seg, img, m), want)
    finally:
        seg.set_diag(False)
    assert np.array_equal(gpu_ws(seg, img, m), want)
