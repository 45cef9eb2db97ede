"""Where a speculative generation's cascade pops spend their time (diagnostic build only:
libmsegment built with -DMSEG_SPEC_PROF, selected through MSEGMENT_LIB).  Per input: rounds,
executions per pop, and for the cascade pops inside k_spec_round the lane-summed s_memtime cycles
of queue selection (the per-lane LDS queue scan + shift), the loads (weights + the four neighbour
views) and the writes (claims, labels, records), with the average queue length scanned.
usage: MSEGMENT_LIB=.../libmsegment_specprof.so python scripts/spec_phases.py mosaic_noise_1024_s1 ..."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "opencv-msegment_amd")]

import torch  # noqa: E402

import msegment  # noqa: E402
from msegment import synth  # noqa: E402


def main():
    seg = msegment.Segmenter(0)
    dev = torch.device("cuda", 0)
    for nm in sys.argv[1:]:
        kind, S, seed = nm.rsplit("_", 2)
        S = int(S)
        img, m, _ = synth.frame(kind, S, S, int(seed[1:]))
        ti, tm = torch.from_numpy(img).to(dev), torch.from_numpy(m).to(dev)
        tl = torch.empty_like(tm)
        seg.watershed_dev(ti, tm, tl)
        torch.cuda.synchronize()
        seg.set_diag(3)
        seg.watershed_dev(ti, tm, tl)
        torch.cuda.synchronize()
        st = seg.stats()
        seg.set_diag(False)
        d = st["diag"]
        n = max(1, d[0])
        tot = max(1, d[2] + d[3] + d[4])
        print("%s: gens %d rounds %d execs/pop %.2f (replayed %.2f) | cascade pops (lane sums) %d, avg queue %.2f | cycles per cascade pop:"
              " select %.0f (%.0f%%), loads %.0f (%.0f%%), writes %.0f (%.0f%%) | wave-cooperative pops %d, %.0f cycles each" % (
                  nm, st["spec_generations"], st["spec_rounds"], st["spec_executions"] / max(1, st["pops"]),
                  st["spec_replays"] / max(1, st["pops"]), d[0],
                  d[1] / n, d[2] / n, 100.0 * d[2] / tot, d[3] / n, 100.0 * d[3] / tot, d[4] / n, 100.0 * d[4] / tot,
                  d[5], d[6] / max(1, d[5])),
              flush=True)
        # the wave-cooperative pop's phases (diag bank 3, s_memtime cycles summed over pops)
        seg.set_diag(4)
        seg.watershed_dev(ti, tm, tl)
        torch.cuda.synchronize()
        st3 = seg.stats()
        seg.set_diag(False)
        c = st3["diag"]
        tot3 = max(1, sum(c[:5]))
        print("%s: cooperative pop phases (cycles per pop over %d pops): loads issued + queue fix %.0f, wait for"
              " the loads %.0f, writes + decision %.0f, pushes %.0f, select %.0f (%.0f%% waiting)" % (
                  nm, d[5], c[0] / max(1, d[5]), c[1] / max(1, d[5]), c[2] / max(1, d[5]), c[3] / max(1, d[5]),
                  c[4] / max(1, d[5]), 100.0 * c[1] / tot3), flush=True)
        # wall-clock split of the round kernels (diag bank 1, 10 ns ticks): wave time in top-pop
        # waits / cascades / whole kernel, and the sum over rounds of each round's longest wave
        seg.set_diag(1)
        torch.cuda.synchronize()
        t0 = torch.cuda.Event(enable_timing=True)
        t1 = torch.cuda.Event(enable_timing=True)
        t0.record()
        seg.watershed_dev(ti, tm, tl)
        t1.record()
        torch.cuda.synchronize()
        st = seg.stats()
        seg.set_diag(False)
        d = st["diag"]
        w = max(1, d[7])
        print("%s: flood %.1f ms (diag on) | waves %d, %.1f us each | sum of the rounds' longest waves %.1f ms over"
              " %d rounds (%.1f us/round): cooperative cascades %.1f ms, top-pop waits %.1f ms, top-pop writes +"
              " cascades %.1f ms, log copy + change marks %.1f ms" % (
                  nm, t0.elapsed_time(t1), d[7], d[2] / w / 100, d[5] / 1e5, st["spec_rounds"],
                  d[5] / 100 / max(1, st["spec_rounds"]), d[0] / 1e5, d[4] / 1e5, d[6] / 1e5, d[1] / 1e5), flush=True)
    seg.close()


if __name__ == "__main__":
    main()
