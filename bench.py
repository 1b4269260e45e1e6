#!/usr/bin/env python3
"""Benchmark: BASELINE.json metric — Msamples/s (+ Mrays/s) of the Cornell-box path tracer,
PathIntegrator depth 8, 1920x1080 x 64 spp (BASELINE config C2; C3 when launched on N GPUs).

One "step" = one full frame (132.7 M camera samples) rendered through the C API
(yafaray_amd_renderQuiet = yafaray_render without the per-pixel callbacks), inputs resident on
the GPU.  On N GPUs (torch.distributed.run, one process per GPU, backend nccl = RCCL) the frame's
32-pixel tile rows are dealt round-robin to the ranks and the finished tile rows are all-gathered
over RCCL into the full film every step (strong scaling: total work fixed).

Prints ONE JSON line (rank 0).  Extra keys: mrays_per_s, roofline (k_trace vs HBM), cpu_baseline
(the CPU oracle restatement on the host cores, bounded sample of the same frame).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mrays/sec + Msamples/sec, 1920×1080×64spp path-trace at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
LDS_PEAK_GBS = 256 * 256 * 2.4   # 256 CUs x 256 B/clk (ds_read_b128, MI355X_MICROARCH.md §LDS) x 2.4 GHz
VALU_PEAK_GIPS = 256 * 4 * 2.4 / 2   # wave64 VALU instructions: 4 SIMD-32 per CU, 2 cycles each (MI355X_MICROARCH.md)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--spp", type=int, default=None, help="default 64 (C2/C4), 1 (C5 photon)")
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--no-rr", action="store_true", help="Russian roulette off (bit-parity variant)")
    ap.add_argument("--scene", default="cornell", choices=["cornell", "sphere", "photon"])
    ap.add_argument("--photons", type=int, default=10_000_000, help="C5: diffuse photons")
    ap.add_argument("--chunk", type=int, default=1 << 26)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    return ap.parse_args()


def workload_name(a, W, H):
    if a.scene == "photon":
        return (f"C5 Cornell PhotonIntegrator, {a.photons} diffuse photons, k=50 gather r^2=0.1, finalGather off, "
                f"{W}x{H}x{a.spp}spp (photon map rebuilt every step)")
    return (f"C2 Cornell PathIntegrator depth {a.bounces}, {W}x{H}x{a.spp}spp"
            + (", RR off" if a.no_rr else ", RR on (reference default)")
            + ("" if a.scene == "cornell" else " + 1M-triangle sphere (C4)"))


def traffic_config(a, W, H):
    return f"{a.scene}-{W}x{H}x{a.spp}-b{a.bounces}-rr{int(not a.no_rr)}-chunk{a.chunk}"


def main():
    a = parse()
    if a.spp is None:
        a.spp = 1 if a.scene == "photon" else 64
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    import torch
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local_rank)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local_rank))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())

    import libyafaray_amd as Y
    from libyafaray_amd import scenes, tiles
    if a.scene == "sphere":
        spec = scenes.cornell_sphere(width=a.width, height=a.height, spp=a.spp, bounces=a.bounces, rr=not a.no_rr)
    elif a.scene == "photon":
        spec = scenes.cornell_photon(a.width, a.height, spp=a.spp, photons=a.photons)
    else:
        spec = scenes.cornell(a.width, a.height, spp=a.spp, bounces=a.bounces, rr=not a.no_rr)
    # the reference's PathIntegrator default caustic_type is "path" (integrator_path_tracer.cc:43);
    # a diffuse-only scene never takes a caustic branch either way.
    yi = Y.Interface()
    scenes.apply(spec, yi)
    yi.L.yafaray_amd_setChunkSlots(yi.h, a.chunk)
    # one contiguous pixel-row band per rank (+ its halo row): equal rows at first, then the
    # boundaries follow the ranks' measured render times (tiles.rebalance_bands, every step)
    if not yi.L.yafaray_amd_buildAccelerator(yi.h):
        raise RuntimeError(yi.last_error())

    W, H = a.width, a.height
    bounds = [tiles.band_range(H, r, world)[0] for r in range(world)] + [H]
    max_rows = min(H, -(-H * 5 // (4 * world)) + 1)    # a band may grow to 1.25x the mean
    band = torch.zeros((max_rows, W, 4), dtype=torch.float32, device=dev)
    gathered = torch.zeros((world * max_rows, W, 4), dtype=torch.float32, device=dev) if world > 1 else None
    t_all = torch.zeros(world, dtype=torch.float64, device=dev) if world > 1 else None

    def step():
        y0, y1 = bounds[rank], bounds[rank + 1]
        yi.L.yafaray_amd_setRowBandRange(yi.h, y0, y1, world)
        t_r = time.perf_counter()
        yi.render_quiet()
        t_r = time.perf_counter() - t_r
        if y1 > y0 and not yi.L.yafaray_amd_getFilmDevice(yi.h, band.data_ptr(), y0, y1):
            raise RuntimeError(yi.last_error())
        if world > 1:
            dist.all_gather_into_tensor(gathered, band)
            dist.all_gather_into_tensor(t_all, torch.tensor([t_r], dtype=torch.float64, device=dev))
            bounds[:] = tiles.rebalance_bands(bounds, t_all.tolist(), cap_rows=max_rows)

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        step()
    # timed region: k_trace launches bracketed by HIP events on the render stream (profile mode)
    yi.L.yafaray_amd_setProfileKernels(yi.h, 1)
    sync()
    t0 = time.perf_counter()
    stats_acc = []
    for _ in range(a.steps):
        step()
        stats_acc.append(yi.stats())
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([sum(s["closest_rays"] + s["shadow_rays"] for s in stats_acc),
                            sum(s["node_visits"] for s in stats_acc), sum(s["tri_tests"] for s in stats_acc)],
                           device=dev, dtype=torch.float64)
        dist.all_reduce(tot)
        rays_total = float(tot[0].item())
    else:
        rays_total = float(sum(s["closest_rays"] + s["shadow_rays"] for s in stats_acc))

    samples_total = float(W * H * a.spp * a.steps)     # whole job: every rank's tile rows together
    msps = samples_total / elapsed / 1e6
    mrays = rays_total / elapsed / 1e6

    # roofline of the dominant kernel (k_trace) on this rank, per launch, with the average launch
    # duration from HIP events on the render stream.  Algorithmic bytes:
    #   ray I/O      closest 32 B in + 8 B out, shadow 32 B in + 4 B index + 1 B out  (always HBM)
    #   traversal    64 B (BVH2) / 128 B (BVH4) per BVH node visited + 48 B per triangle tested
    # The traversal bytes count against HBM only when the scene is not LDS-resident; for the
    # Cornell box (3 KB) they are served by LDS and reported separately against the LDS peak.
    s = stats_acc[-1]
    launches = max(1, s["trace_launches"])
    avg_ms = s["trace_kernel_ms"] / launches
    ray_io = 40.0 * s["closest_rays"] + 37.0 * s["shadow_rays"]
    node_bytes = 128.0 if s["bvh_width"] == 4 else 64.0
    trav = node_bytes * s["node_visits"] + 48.0 * s["tri_tests"]
    in_lds = bool(s["scene_in_lds"])
    algo_bytes = ray_io + (0.0 if in_lds else trav)
    per_launch = algo_bytes / launches
    achieved = per_launch / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    trav_rate = trav / launches / (avg_ms * 1e-3) / 1e9 if avg_ms > 0 else 0.0
    traffic = None
    valu_insts = None
    tfile = os.path.join(ROOT, "profiles", "trace_hbm_bytes_per_launch.json")
    if os.path.exists(tfile):
        try:
            with open(tfile) as f:
                tj = json.load(f)
            import hashlib
            with open(os.path.join(ROOT, "libyafaray_amd", "csrc", "kernels.hip"), "rb") as f:
                sha = hashlib.sha1(f.read()).hexdigest()
            # only a measurement of this exact kernel source on this exact workload counts
            if tj.get("config") == traffic_config(a, W, H) and tj.get("kernels_hip_sha1") == sha:
                traffic = tj.get("hbm_bytes_per_launch")
                valu_insts = tj.get("valu_insts_per_launch")
        except Exception:
            traffic = None

    cpu = None
    if rank == 0 and world == 1 and not a.no_cpu_baseline:
        cpu = cpu_baseline(spec, a)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(msps, 3),
            "unit": "Msamples/s",
            "n_gpus": world,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Cornell box scene generated in-repo, SURVEY.md §8d)",
            "config": {"workload": workload_name(a, W, H),
                       "width": W, "height": H, "spp": a.spp, "bounces": a.bounces,
                       "samples_per_step": W * H * a.spp, "parallelism": f"row-bands x{world}",
                       "chunk_slots": a.chunk},
            "mrays_per_s": round(mrays, 2),
            "rays_per_sample": round(rays_total / samples_total, 3),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                         "kernel": "k_trace", "avg_launch_ms": round(avg_ms, 4), "launches_per_step": launches,
                         "algo_bytes_per_launch": round(per_launch),
                         # VALU issue (the bound of an LDS-resident traversal): PMC SQ_INSTS_VALU per launch
                         # (same kernels.hip + workload only) / the live launch time, against 256 CUs x 4 SIMDs
                         # x 2.4 GHz / 2 cycles per wave64 VALU instruction
                         "valu": ({"insts_per_launch": valu_insts,
                                   "achieved_g_per_s": round(valu_insts / (avg_ms * 1e-3) / 1e9, 1),
                                   "peak_g_per_s": VALU_PEAK_GIPS,
                                   "frac": round(valu_insts / (avg_ms * 1e-3) / 1e9 / VALU_PEAK_GIPS, 4)}
                                  if valu_insts and avg_ms > 0 else None),
                         "traversal": {"bytes_per_launch": round(trav / launches), "served_from": "LDS" if in_lds else "L2/MALL/HBM",
                                       "achieved": round(trav_rate, 1), "unit": "GB/s",
                                       "lds_peak": LDS_PEAK_GBS, "frac_of_lds_peak": round(trav_rate / LDS_PEAK_GBS, 4),
                                       "bvh_width": s["bvh_width"],
                                       "node_visits_per_ray": round(s["node_visits"] / max(1, s["closest_rays"] + s["shadow_rays"]), 2),
                                       "tri_tests_per_ray": round(s["tri_tests"] / max(1, s["closest_rays"] + s["shadow_rays"]), 2)}},
            "shade": {"avg_launch_ms": round(s["shade_kernel_ms"] / launches, 4),
                      "ms_per_step": round(s["shade_kernel_ms"], 2), "trace_ms_per_step": round(s["trace_kernel_ms"], 2),
                      "nee_ms_per_step": round(s["nee_kernel_ms"], 2)},
            "photon_map": ({"photons_stored": s["photons"], "seconds_per_step": round(s["photon_seconds"], 4),
                            "shoot_seconds": round(s["photon_shoot_seconds"], 4), "tree_seconds": round(s["photon_tree_seconds"], 4)}
                           if a.scene == "photon" else None),
            "launch": {k: s[k] for k in ("trace_grid", "shade_grid", "trace_block", "stack_depth", "scene_in_lds", "bvh_nodes")},
            # accelerator build + scene upload, once before the timed region (the reference builds
            # its kd-tree inside render(), scene.cc:218)
            "scene_build_seconds": round(s["build_seconds"], 4),
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    yi.close()
    if world > 1:
        dist.destroy_process_group()


def cpu_baseline(spec, a):
    """The CPU oracle (C++ restatement of the reference loop) on the host cores, on a bounded
    band of rows of the same frame, scaled to Msamples/s."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}
    cores = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or min(16, os.cpu_count() or 1)
    cores = max(1, min(cores, os.cpu_count() or 1))
    photon_note = ""
    t_photons = 0.0
    if spec.render.integrator == "photonmapping":
        # C5: the oracle shoots and builds single-threaded; time a tenth of the photons and scale
        # linearly (optimistic for the n log n tree), then render a row band with that map.
        import dataclasses
        n_full = spec.render.pm_photons
        n_cpu = max(1000, n_full // 10)
        spec = dataclasses.replace(spec, render=dataclasses.replace(spec.render, pm_photons=n_cpu))
        t0 = time.perf_counter()
        O.OracleScene(spec, threads=1).photon_map()
        t_photons = (time.perf_counter() - t0) * (n_full / n_cpu)
        photon_note = f"; photon map: {n_cpu} photons shot+built in {t_photons * n_cpu / n_full:.1f} s (1 thread), scaled x{n_full / n_cpu:g}"
    osc = O.OracleScene(spec, threads=cores)
    # probe one 32-row tile band, then size the sample to ~cpu_seconds
    ts = spec.render.tile_size
    y0 = (spec.render.height // 2 // ts) * ts
    t0 = time.perf_counter()
    osc.render(y0, y0 + 4)
    probe = time.perf_counter() - t0
    per_row = probe / 4
    rows = int(max(4, min(spec.render.height - y0, a.cpu_seconds / max(per_row, 1e-6))))
    t0 = time.perf_counter()
    _, _, ctr = osc.render(y0, y0 + rows)
    dt = time.perf_counter() - t0
    n = rows * spec.render.width * spec.render.aa_samples
    if t_photons > 0.0:
        # whole frame = photon map + every row; rate over the frame
        frame = spec.render.width * spec.render.height * spec.render.aa_samples
        t_frame = t_photons + dt * frame / n
        return {"value": round(frame / t_frame / 1e6, 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
                "sample": f"rows {y0}..{y0 + rows} of the {spec.render.width}x{spec.render.height} frame "
                          f"({n} samples, {dt:.1f} s, {cores} threads){photon_note}"}
    return {"value": round(n / dt / 1e6, 4), "unit": "Msamples/s", "cores": cores, "kind": "port",
            "mrays_per_s": round((ctr[0] + ctr[1]) / dt / 1e6, 3),
            "sample": f"rows {y0}..{y0 + rows} of the same {spec.render.width}x{spec.render.height}x"
                      f"{spec.render.aa_samples}spp frame ({n} samples, {dt:.1f} s, {cores} threads)"}


if __name__ == "__main__":
    main()
