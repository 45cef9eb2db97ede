"""The interrupt-dense regime per frame: flood time, the speculative engine's counters (generations,
rounds, executions, cascade pops, fallbacks, cooldowns, the pops generations committed and their
device time) and, optionally, the same frame with the engine off and the C oracle's time.
Frames are named kind_S_sSEED (synth.frame), or album_shape / album_color (album.jpg with the
shape / colour method's seeds).  usage: python scripts/spec_probe.py [--oracle] [--off] NAME..."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def load(seg, nm):
    if nm.startswith("album"):
        from PIL import Image
        rgb = np.asarray(Image.open(os.path.join(ROOT, "tests", "golden", "album_1500x1500.png")).convert("RGB"))
        album = np.ascontiguousarray(rgb[..., ::-1])
        if nm == "album_color":
            sharp, mk, _ = seg.color_markers(album)
            return np.ascontiguousarray(sharp), np.ascontiguousarray(mk)
        return album, np.ascontiguousarray(seg.shape_markers(album)[0])
    nc = nm.startswith("nc_")
    kind, S, seed = (nm[3:] if nc else nm).rsplit("_", 2)
    img, m, _ = synth.frame(kind, int(S), int(S), int(seed[1:]))
    if nc:
        m = np.ascontiguousarray(seg.nc_marker_stage(img, 4)[0])
    return img, m


def flood_ms(seg, ti, tm, tl, reps=1):
    seg.watershed_dev(ti, tm, tl)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        seg.watershed_dev(ti, tm, tl)
    torch.cuda.synchronize()
    return 1e3 * (time.perf_counter() - t0) / reps


def main():
    args = sys.argv[1:]
    do_oracle = "--oracle" in args
    do_off = "--off" in args
    names = [a for a in args if not a.startswith("--")]
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for nm in names:
        img, m = load(seg, nm)
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        ms = flood_ms(seg, ti, tm, tl)
        st = seg.stats()
        px = m.size
        line = ("%-22s %9.1f ms %8.2f Mpx/s | pops %d batches %d | gens %d rounds %d execs/pop %.2f cpops %d "
                "fallbacks %d cools %d replays %d gen_pops %d gen_ms %.1f xpops %d longest %d" % (
                    nm, ms, px / ms / 1e3, st["pops"], st["batches"], st["spec_generations"], st["spec_rounds"],
                    st["spec_executions"] / max(1, st["pops"]), st["spec_cascade_pops"], st["spec_fallbacks"],
                    st["spec_cooldowns"], st["spec_replays"], st["spec_gen_pops"], st["spec_gen_us"] / 1e3,
                    st["spec_exec_pops"], st["spec_longest_pops"]))
        ok = ""
        if do_oracle:
            from oracle import ws_oracle
            c0 = time.perf_counter()
            want = ws_oracle.watershed(img, m)
            cms = 1e3 * (time.perf_counter() - c0)
            ok = " | oracle %.1f ms %s" % (cms, "bit-exact" if np.array_equal(tl.cpu().numpy(), want) else "MISMATCH")
        if do_off:
            seg.set_speculative(False)
            ok += " | engine off %.1f ms" % flood_ms(seg, ti, tm, tl)
            seg.set_speculative(True)
        print(line + ok, flush=True)
    seg.close()


if __name__ == "__main__":
    main()
