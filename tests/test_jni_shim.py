"""The JNI shim (opencv-msegment_amd/jni/msegment_jni.cpp) compiled and driven without a JDK:
tests/jni_stub/jni.h declares the JNI subset it uses with the JDK's types and signatures, and
tests/jni_stub/mock_env.cpp implements them over std::vectors (bounds-checked region copies,
counted critical regions).  CPU: every short / negative / oversized argument returns MSG_EINVAL
before the library is touched.  GPU: one PictureService.watershed call through the shim against
the oracle."""
import os
import struct
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUB = os.path.join(ROOT, "tests", "jni_stub")
LIBDIR = os.path.join(ROOT, "opencv-msegment_amd", "msegment")


def build(tmp_path):
    exe = str(tmp_path / "mock_env")
    cmd = ["g++", "-std=c++17", "-O1", "-Wall", "-Werror", "-I", STUB, "-I", os.path.join(ROOT, "include"),
           os.path.join(ROOT, "opencv-msegment_amd", "jni", "msegment_jni.cpp"), os.path.join(STUB, "mock_env.cpp"),
           "-L", LIBDIR, "-lmsegment", "-Wl,-rpath," + LIBDIR, "-o", exe]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def test_jni_shim_compiles_and_validates(tmp_path):
    if not os.path.exists(os.path.join(LIBDIR, "libmsegment.so")):
        pytest.skip("libmsegment.so not built (run __graft_entry__.build())")
    exe = build(tmp_path)
    r = subprocess.run([exe, "validate"], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "validate ok" in r.stdout


@pytest.mark.gpu
def test_jni_shim_watershed_on_gpu(tmp_path):
    from msegment import synth
    from msegment.jrandom import generate_bgr_palette
    from oracle import ws_oracle

    exe = build(tmp_path)
    img, m, d = synth.frame("mosaic_noise", 120, 90, 5)
    pal = generate_bgr_palette(d, 7)
    src, dst = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    with open(src, "wb") as f:
        f.write(struct.pack("<4i", 120, 90, d, 1))
        f.write(img.tobytes())
        f.write(m.astype(np.int32).tobytes())
        f.write(np.ascontiguousarray(pal, dtype=np.uint8).tobytes())
    r = subprocess.run([exe, "run", src, dst], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(dst, "rb").read()
    rc = struct.unpack("<i", raw[:4])[0]
    assert rc == 0
    n = 120 * 90
    lab = np.frombuffer(raw[4:4 + 4 * n], np.int32).reshape(120, 90)
    out = np.frombuffer(raw[4 + 4 * n:], np.uint8).reshape(120, 90, 3)
    want = ws_oracle.watershed(img, m)
    assert np.array_equal(lab, want)
    assert np.array_equal(out, ws_oracle.colorize(want, d, pal))


@pytest.mark.gpu
@pytest.mark.parametrize("mode,devs", [(0, None), (1, None), (0, "0,0"), (1, "0,0")])
def test_jni_shim_batch_on_gpu(tmp_path, mode, devs):
    """MSegmentNative.watershedColorizeBatch through the shim: CorrelationTestService's many floods
    per image (CorrelationTestService.java:84-86, 141 -> PictureService.java:852) handed over in one
    call, in the default batch path (mode 0) and the many-floods mode (mode 1); with devs, spread
    over the device list {0, 0} first (MSegmentNative.watershedBatch(..., devices) ->
    setBatchDevices -> msg_set_batch_devices: two sub-contexts, frames 0-1 and 2-4)."""
    from msegment import synth
    from msegment.jrandom import generate_bgr_palette
    from oracle import ws_oracle

    exe = build(tmp_path)
    rng = np.random.default_rng(11)
    frames = []
    for k, (H, W) in enumerate(((96, 128), (64, 64), (0, 7), (130, 70), (33, 41))):
        img = synth.frame("mosaic_noise", max(H, 1), max(W, 1), 20 + k)[0][:H, :W]
        m = np.where(rng.random((H, W)) < 0.03, rng.integers(1, 6, (H, W)), 0).astype(np.int32)
        frames.append((np.ascontiguousarray(img), m))
    depth = 5
    pal = generate_bgr_palette(depth, 3)
    src, dst = str(tmp_path / "in.bin"), str(tmp_path / "out.bin")
    with open(src, "wb") as f:
        f.write(struct.pack("<3i", len(frames), depth, 1))
        f.write(np.ascontiguousarray(pal, dtype=np.uint8).tobytes())
        for img, m in frames:
            f.write(struct.pack("<2i", *m.shape))
            f.write(img.tobytes())
            f.write(m.tobytes())
    r = subprocess.run([exe, "batch", str(mode), src, dst] + ([devs] if devs else []), capture_output=True,
                       text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    raw = open(dst, "rb").read()
    assert struct.unpack("<i", raw[:4])[0] == 0
    off = 4
    for img, m in frames:
        n = m.size
        lab = np.frombuffer(raw[off:off + 4 * n], np.int32).reshape(m.shape)
        off += 4 * n
        out = np.frombuffer(raw[off:off + 3 * n], np.uint8).reshape(m.shape + (3,))
        off += 3 * n
        want = ws_oracle.watershed(img, m)
        assert np.array_equal(lab, want)
        assert np.array_equal(out, ws_oracle.colorize(want, depth, pal))
