"""Per-rank render time of the C2 frame split over WORLD GPUs, rehearsed on one GPU (each rank's
share rendered in turn): predicts the strong-scaling efficiency of bench.py --gpus WORLD.

    python tools/shard_probe.py [WORLD ...] [--mode band|tile]
"""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import libyafaray_amd as Y  # noqa: E402
from libyafaray_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("worlds", nargs="*", type=int, default=[1, 2, 4, 8])
    ap.add_argument("--mode", default="band", choices=["band", "tile"])
    ap.add_argument("--reps", type=int, default=2)
    a = ap.parse_args()
    spec = scenes.cornell(1920, 1080, spp=64, bounces=8, rr=True)
    yi = Y.Interface()
    scenes.apply(spec, yi)
    yi.L.yafaray_amd_setChunkSlots(yi.h, 1 << 25)
    if not yi.L.yafaray_amd_buildAccelerator(yi.h):
        raise RuntimeError(yi.last_error())
    t1 = None
    for world in a.worlds:
        times = []
        for r in range(world):
            fn = yi.L.yafaray_amd_setRowBandShard if a.mode == "band" else yi.L.yafaray_amd_setTileRowShard
            fn(yi.h, r, world)
            yi.render_quiet()   # warm
            best = 1e9
            for _ in range(a.reps):
                t0 = time.perf_counter()
                yi.render_quiet()
                best = min(best, time.perf_counter() - t0)
            times.append(best)
        tmax = max(times)
        if world == 1:
            t1 = tmax
        eff = (t1 / (world * tmax)) if t1 else float("nan")
        print(f"world {world} ({a.mode}): per-rank ms min {1e3 * min(times):.1f} max {1e3 * tmax:.1f} "
              f"-> predicted efficiency {eff:.3f}", flush=True)
    yi.close()


if __name__ == "__main__":
    main()
