"""GPU: the batch entry points' many-floods mode (msg_set_batch_floods: every frame of the call in
one k_serial_multi launch, one wave per flood) against the C oracle, frame by frame.  The frames
are the serial regime the mode is for -- scattered notConnectedMarkers-style seeds, uniform noise,
an album.jpg crop with the shape method's seeds -- plus a plateau mosaic (mode 2 hands it back to
the full engine) and degenerate sizes."""
import os

import numpy as np
import pytest

from msegment import synth
from oracle import ws_oracle

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def frames():
    out = []
    for kind, H, W, seed in (("random", 96, 128, 1), ("mosaic_noise", 128, 128, 2), ("mosaic", 160, 96, 3),
                             ("random", 3, 3, 4), ("random", 1, 7, 5), ("mosaic_noise", 61, 257, 6)):
        img, m, _ = synth.frame(kind, H, W, seed)
        out.append((img, m))
    rng = np.random.default_rng(7)
    img = synth.frame("mosaic_noise", 200, 200, 8)[0]
    m = np.where(rng.random((200, 200)) < 0.02, rng.integers(1, 9, (200, 200)), 0).astype(np.int32)
    out.append((img, m))  # scattered seeds with few labels: the NC pipeline's kind of markers
    from PIL import Image
    rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
    album = np.ascontiguousarray(rgb[200:456, 300:620, ::-1])
    m = np.zeros(album.shape[:2], np.int32)
    m[::37, ::41] = np.arange(1, m[::37, ::41].size + 1).reshape(m[::37, ::41].shape)
    out.append((album, m))
    # zero-pixel frames between the others (round 4's advisor: a 0 x W / H x 0 flood has no
    # workspace, and k_serial_multi used to read its null control block)
    out.insert(2, (np.zeros((0, 9, 3), np.uint8), np.zeros((0, 9), np.int32)))
    out.append((np.zeros((5, 0, 3), np.uint8), np.zeros((5, 0), np.int32)))
    return out


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_batch_many_host_buffers(seg, mode):
    fr = frames()
    work = [m.copy() for _, m in fr]
    seg.set_batch_floods(mode)
    try:
        seg.watershed_batch([(img, w) for (img, _), w in zip(fr, work)])
    finally:
        seg.set_batch_floods(0)  # releases the workspaces; back to the default (automatic) mode
        seg.set_batch_floods(3)
    for k, ((img, m), got) in enumerate(zip(fr, work)):
        assert np.array_equal(got, ws_oracle.watershed(img, m)), k


@pytest.mark.parametrize("mode", [1, 2, 3])
def test_batch_many_device(seg, mode):
    import torch

    dev = torch.device("cuda", seg.device)
    fr = frames()
    depth = 64
    imgs = [torch.from_numpy(img).to(dev) for img, _ in fr]
    mks = [torch.from_numpy(m).to(dev) for _, m in fr]
    labs = [torch.empty_like(x) for x in mks]
    dsts = [torch.empty(img.shape, dtype=torch.uint8, device=dev) for img, _ in fr]
    seg.set_batch_floods(mode)
    try:
        seg.watershed_colorize_batch_dev(imgs, mks, labs, depth, None, dsts)
    finally:
        seg.set_batch_floods(0)  # releases the workspaces; back to the default (automatic) mode
        seg.set_batch_floods(3)
    torch.cuda.synchronize()
    for k, (img, m) in enumerate(fr):
        want = ws_oracle.watershed(img, m)
        assert np.array_equal(labs[k].cpu().numpy(), want), k
        assert np.array_equal(dsts[k].cpu().numpy(), ws_oracle.colorize(want, depth, None)), k
        assert np.array_equal(mks[k].cpu().numpy(), m), k  # inputs untouched


def test_batch_many_repeat_and_grow(seg):
    """Two calls in a row on the same context (workspaces reused), the second with more frames."""
    fr = frames()
    seg.set_batch_floods(1)
    try:
        for n in (3, len(fr)):
            work = [m.copy() for _, m in fr[:n]]
            seg.watershed_batch([(img, w) for (img, _), w in zip(fr[:n], work)])
            for k in range(n):
                assert np.array_equal(work[k], ws_oracle.watershed(*fr[k])), (n, k)
    finally:
        seg.set_batch_floods(0)  # releases the workspaces; back to the default (automatic) mode
        seg.set_batch_floods(3)


def test_auto_mode_probe_and_choice(seg):
    """msg_set_batch_floods 3 (the default): the first call of a frame size floods frame 0 alone
    (batch_probe) and picks the path; the next call of that size reuses the choice without a probe.
    Plateau mosaics price far below a serial pop per pixel and stay on the full engine (mode 0);
    scattered seeds on a textured frame (notConnectedMarkers' kind) take whichever path the probe
    prices lower -- every frame bit-exact either way, host and device entry points."""
    import torch

    dev = torch.device("cuda", seg.device)
    seg.set_batch_floods(3)
    mos = [synth.frame("mosaic", 512, 512, 40 + k)[:2] for k in range(6)]
    for call in range(2):
        work = [m.copy() for _, m in mos]
        seg.watershed_batch([(img, w) for (img, _), w in zip(mos, work)])
        st = seg.stats()
        assert st["batch_mode"] == 0 and st["batch_probe"] == (1 if call == 0 else 0), (call, st["batch_mode"])
        for (img, m), got in zip(mos, work):
            assert np.array_equal(got, ws_oracle.watershed(img, m))
    rng = np.random.default_rng(5)
    scat = []
    for k in range(12):
        img = synth.frame("mosaic_noise", 256, 256, 60 + k)[0]
        m = np.where(rng.random((256, 256)) < 0.02, rng.integers(1, 6, (256, 256)), 0).astype(np.int32)
        scat.append((img, m))
    imgs = [torch.from_numpy(img).to(dev) for img, _ in scat]
    mks = [torch.from_numpy(m).to(dev) for _, m in scat]
    labs = [torch.empty_like(x) for x in mks]
    dsts = [torch.empty(img.shape, dtype=torch.uint8, device=dev) for img, _ in scat]
    for call in range(2):
        seg.watershed_colorize_batch_dev(imgs, mks, labs, 5, None, dsts)
        torch.cuda.synchronize()
        st = seg.stats()
        assert st["batch_mode"] in (0, 1) and st["batch_probe"] == (1 if call == 0 else 0)
        for k, (img, m) in enumerate(scat):
            assert np.array_equal(labs[k].cpu().numpy(), ws_oracle.watershed(img, m)), (call, k)
    print("scattered seeds 256^2 x 12: automatic mode chose", st["batch_mode"])
    seg.set_batch_floods(0)
    seg.set_batch_floods(3)
