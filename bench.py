#!/usr/bin/env python3
"""Benchmark: BASELINE.json metric — Msamples/s (+ Mrays/s) of the Cornell-box path tracer,
PathIntegrator depth 8, 1920x1080 x 64 spp (BASELINE config C2; C3 when launched on N GPUs).

One "step" = one full frame (132.7 M camera samples) rendered through the C API
(yafaray_amd_renderQuiet = yafaray_render without the per-pixel callbacks), inputs resident on
the GPU.  On N GPUs every member renders one contiguous band of pixel rows and the library itself
combines the bands (the multi-GPU split lives behind the drop-in boundary):
  * torch.distributed.run, one process per GPU (WORLD_SIZE = N): a render group
    (yafaray_amd_setRenderGroup), bands all-gathered over RCCL into every rank's film;
  * `python bench.py --gpus N` in one process: a device group (yafaray_amd_setDeviceGroup, what an
    unmodified client gets from the "gpus" render parameter), one host thread + stream per GPU,
    member 0 pulls the bands over xGMI.

Prints ONE JSON line (rank 0).  Extra keys:
  * mrays_per_s                       closest + shadow rays per second (in-kernel counters)
  * roofline                          the dominant kernel against its bound (HIP events live, per launch)
  * kernels                           every kernel: time share, algorithmic bytes per work item
                                      (SURVEY §8d model), measured HBM traffic (PMC,
                                      profiles/pmc_<config>.json), achieved GB/s and fraction of 8 TB/s
  * parity                            full-size checks of this frame against the CPU oracle:
                                      the cpu_baseline band (RR on: paired z of the difference
                                      image's 8x8 block means, oracle/stats.py, for two RR seeds)
                                      and an RR-off band bit for bit
  * cpu_baseline                      the oracle restatement on this host's cores, bounded band
  * build                             sha256 of libyafaray4.so and its compile flags (yafaray_amd_buildInfo)
  * group (N > 1)                     the library's report of the split: devices, peer-access matrix,
                                      band copy path, band bounds, each member's render ms
With N > 1 GPUs `parity` is group_parity's (always run): the group's frame bit for bit against a
one-member render, and an RR-off group frame against the oracle on rows around the band boundaries;
the process exits with status 3 when either differs.
"""
import argparse
import dataclasses
import json
import os
import platform
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402

METRIC = "Mrays/sec + Msamples/sec, 1920×1080×64spp path-trace at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0   # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec
# bytes a traversal visit reads per node: BVH2 64, BVH4 128, quantised BVH8 80 (the first 80 B of its 128-B node)
NODE_BYTES = {2: 64.0, 4: 128.0, 8: 80.0}
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
    ap.add_argument("--scene", default="cornell", choices=["cornell", "sphere", "photon", "meshlight"],
                    help="meshlight: C2 with a 10082-face double-sided meshlight sphere next to the area light (frame time of the meshlight BVH)")
    ap.add_argument("--photons", type=int, default=10_000_000, help="C5: diffuse photons")
    ap.add_argument("--fg", type=int, default=0, help="C5 variant: PhotonIntegrator final gathering with this many fg_samples (0: off, as C5)")
    ap.add_argument("--chunk", type=int, default=1 << 27)
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target length of the CPU baseline sample")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-parity", action="store_true", help="skip the full-size parity checks")
    ap.add_argument("--parity-rows", type=int, default=12, help="rows of the RR-off bit-exact band")
    ap.add_argument("--lights", type=int, default=1, help="C2 variant: 2 or 3 lights (scenes.with_extra_lights); multi-light path tracing "
                    "runs the one-thread light-pick count run per pass (YAFARAY_AMD_LIGHT_PICK=hash skips it)")
    ap.add_argument("--flush-steps", type=int, default=2, help="frames timed through yafaray_render with the film flush (ms_per_step_flush)")
    ap.add_argument("--members-per-gpu", type=int, default=1,
                    help="device-group members per GPU (experiment: several logical members on one GPU run on concurrent streams)")
    return ap.parse_args()


def workload_name(a, W, H):
    if a.scene == "photon":
        fg = f"finalGather on ({a.fg} fg_samples, fg_bounces 2)" if a.fg else "finalGather off"
        return (f"C5 Cornell PhotonIntegrator, {a.photons} diffuse photons, k=50 gather r^2=0.1, {fg}, "
                f"{W}x{H}x{a.spp}spp (photon map rebuilt every step)")
    return (f"C2 Cornell PathIntegrator depth {a.bounces}, {W}x{H}x{a.spp}spp"
            + (", RR off" if a.no_rr else ", RR on (reference default)")
            + (f", {a.lights} lights" if a.lights > 1 else "")
            + {"cornell": "", "sphere": " + 1M-triangle sphere (C4)",
               "meshlight": " + 10082-face double-sided meshlight sphere"}[a.scene])


def pmc_config(a, W, H):
    """Key of profiles/pmc_<key>.json (tools/pmc_all.sh): one workload, one kernel source."""
    return f"{a.scene}-{W}x{H}x{a.spp}-b{a.bounces}-rr{int(not a.no_rr)}-chunk{a.chunk}" + (
        f"-ph{a.photons}" if a.scene == "photon" else "") + (f"-fg{a.fg}" if a.scene == "photon" and a.fg else "") + (
        f"-l{a.lights}" if getattr(a, "lights", 1) > 1 else "") + (
        # a member renders a band: its launches are a fraction of the one-GPU launches the PMC file measured
        f"-g{a.gpus}" if getattr(a, "gpus", 1) > 1 else "") + (
        f"-m{a.members_per_gpu}" if getattr(a, "members_per_gpu", 1) > 1 else "")


def kernels_src_sha1():
    import hashlib
    h = hashlib.sha1()
    # every source the profiled device code is compiled from (kernels and the headers they inline)
    for f in ("kernels.hip", "pkd.hip", "pkd_kernels.h", "aa.hip", "fgthin.hip", "bvhgpu.hip", "devmath.h", "devscene.h", "texeval.h",
              "photonheap.h"):
        with open(os.path.join(ROOT, "libyafaray_amd", "csrc", f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


def load_pmc(a, W, H):
    """Per-kernel PMC traffic of this exact workload and kernel source, or None."""
    path = os.path.join(ROOT, "profiles", f"pmc_{pmc_config(a, W, H)}.json")
    if not os.path.exists(path):
        return None
    try:
        with open(path) as f:
            pj = json.load(f)
    except Exception:
        return None
    if pj.get("config") != pmc_config(a, W, H) or pj.get("kernels_src_sha1") != kernels_src_sha1():
        return None
    return pj


# ---------------------------------------------------------------------------------------------
# algorithmic bytes per work item (DESIGN.md §4 restates each with our design's bytes)
# ---------------------------------------------------------------------------------------------
# kernel kinds that are one kernel (per-launch PMC instruction counts map onto their launches); the
# others (pkd_build, photon_compact, aa_next_pass) are sequences of several kernels per launch record
# (k_fg: k_fg_first + k_fg_long + k_fg_sum per batch record, r06; k_pregather: k_rad_refl + k_pregather)
SINGLE_KERNEL_KINDS = {"k_trace", "k_shade", "k_nee", "k_camera", "k_film", "k_gather", "k_gather_walk", "k_surface",
                       "k_tshadow", "k_photon_emit", "k_photon_bounce", "k_spawn", "k_combine"}
# SURVEY §8d per-ray algorithmic bytes with the reference kd-tree's measured counts
# (B_ray = N_node * 8 + N_tri * 40 + ray I/O): C2 closest 273 / shadow 235 B, C4 509 / 793 B
SURVEY_B_RAY = {"cornell": (273.0, 235.0), "sphere": (509.0, 793.0)}


def algo_bytes(kind, s, kt, in_lds, a, kt_all=None):
    """Total algorithmic HBM bytes of all launches of one kernel kind in one frame (kt_all: every kind's
    record of the frame, for the models that depend on another kernel's work)."""
    it = kt["items"]
    kt_all = kt_all or {}
    if kind == "k_trace":
        # ray I/O: closest 24 B in (12-B origin + direction records; the camera rays' 8-B (tmin, tmax)
        # ignored) + 8 B out (t, prim); shadow 32 B in (o + index, d + tmax) + 1 B out; traversal bytes
        # (128 B per BVH4 node, 48 B per triangle) only when the scene is not LDS-resident
        trav = NODE_BYTES.get(s["bvh_width"], 64.0) * s["node_visits"] + 48.0 * s["tri_tests"]
        return 32.0 * s["closest_rays"] + 33.0 * s["shadow_rays"] + (0.0 if in_lds else trav)
    if kind == "k_shade":
        return 64.0 * it          # §8d: path-state read + write per path segment
    if kind == "k_nee":
        # per request: the vertex in ((wo, prim) 16 B, the 8-B pixel / sample / mode word, the hit point
        # as the next ray origin 12 B) 36 B;
        # out: one shadow ray per light sample (o + index, d + tmax: 32 B) + contribution (12-B record)
        # + occlusion byte
        return 36.0 * it + 45.0 * (s["shadow_rays"] / max(1, s["closest_rays"])) * it
    if kind == "k_camera":
        # camera ray (12-B origin + direction records) 24 B + the 8-B compact record (sample id + stage; the
        # r05 stateless RR draw keeps no MWC state in it): 32 B per sample, as kernels.hip k_camera writes
        # and PMC WRITE_SIZE measures (32.0 B x samples); a camera entry's zero throughput / colour / flags
        # are implied by its stage (§8d counted 64 B of initial state); the per-ray (tmin, tmax) 8 B only
        # with clip planes (not counted)
        return 32.0 * it
    if kind == "k_film":
        return 16.0 * it + 20.0 * a.width * a.height   # the samples (float4) + RGBA + weight per pixel
    if kind == "k_gather_walk":
        # pass 1 of the two-pass diffuse estimate: §8d's N_visit * 16 B (kd node; a leaf carries the photon
        # position) + 8 B per photon it logs (index + distance) + the request's point (16 B) and its log
        # count (4 B)
        return 16.0 * s.get("gather_visits", 0) + 8.0 * s.get("gather_accepts", 0) + 20.0 * it
    if kind == "k_gather":
        # 36 B per photon record the estimates read (position.w + direction + colour.b, counted in-kernel:
        # under final gathering the diffuse estimate moves to k_fg, so the records are counted, not k per
        # request), plus the request (64 B) and the sample it writes (16 B).  Two-pass gather: the node
        # visits belong to k_gather_walk; this replay reads the walk's log (8 B per logged photon) instead
        walk = kt_all.get("k_gather_walk", {}).get("launches", 0) > 0
        visits = 8.0 * s.get("gather_accepts", 0) if walk else 16.0 * s.get("gather_visits", 0)
        return visits + 36.0 * s.get("gather_photons", 0) + 80.0 * it
    if kind == "k_photon_emit":
        # per photon path: its alive-list slot (4 B) + the path record (origin, direction, colour: 48 B)
        return 52.0 * it
    if kind == "photon_compact":
        # both passes read every deposit slot's flag (1 B each); each stored photon's record is read and
        # written in photon-id order (36 B each way); final gathering: the radiance points' flags likewise
        # and 48 B each way per point
        stored = s.get("photons", 0) + s.get("caustic_photons", 0)
        rad = s.get("radiance_points", 0)
        slots = s.get("photon_slots", 0)
        return 2.0 * slots + 72.0 * stored + ((2.0 * slots + 96.0 * rad) if rad else 0.0)
    if kind == "k_fg":
        # per request: 64 B in (point, wo + sample id, colour, extra) + 16 B out; per radiance-map nearest
        # search the kd nodes it fetched (16 B each, counted in-kernel) and the found point's radiance
        # (three 4-B words of the position / direction / colour arrays, 12 B); per gather path the hit's
        # primitive record (normal + material, 16 B).  The gather rays' traversal bytes count only for a
        # scene in global memory (an LDS-resident scene's never reach HBM)
        return (80.0 * it + 16.0 * s.get("fg_nearest_visits", 0) + 12.0 * s.get("fg_lookups", 0)
                + 16.0 * s.get("fg_paths", 0))
    if kind == "k_photon_bounce":
        # per traced path record (items = paths traced over all bounces): its alive-list slot + origin,
        # direction and colour read (52 B); the paths that continue write the same 52 B (every traced
        # path after bounce 0 was written by the previous bounce, the emitted ones by k_photon_emit);
        # each stored photon's deposit (position, direction, colour.b, flag: 37 B)
        emitted = kt_all.get("k_photon_emit", {}).get("items", 0)
        stored = s.get("photons", 0) + s.get("caustic_photons", 0)
        return 52.0 * it + 52.0 * max(0, it - emitted) + 37.0 * stored
    if kind == "k_pregather":
        # two launches per radiance map: k_rad_refl (per kept point: its 16-B position + primitive read, the
        # two reflectivities written: 16 + 16 + 8 + 16 B) and k_pregather (per kept point: the 48-B point in,
        # the radiance photon out 36 B; the diffuse-map kd nodes it fetched, 16 B each, and the photons it
        # summed, 36 B each — both counted in-kernel)
        return 56.0 * it + 84.0 * it + 16.0 * s.get("pregather_visits", 0) + 36.0 * s.get("pregather_photons", 0)
    if kind == "pkd_build":
        # one launch record per tree: each tree over its own points (the diffuse map, the caustic map, the
        # final-gathering radiance map of the kept points)
        return sum(pkd_build_bytes(n) for n in pkd_trees(s, kt["launches"]))
    return None


def pkd_trees(s, launches):
    """Item counts of the point kd-trees built in one frame (one pkd_build launch record each): the diffuse
    map, then the caustic map and the radiance map when present."""
    trees = [n for n in (s.get("photons", 0), s.get("caustic_photons", 0), s.get("radiance_photons", 0)) if n]
    return trees[:max(1, launches)] if trees else []


def pkd_build_bytes(n):
    """Algorithmic bytes of one point kd-tree build over n photons (pkd.hip): the three presorted
    (coordinate, index) lists — keys 28 B per photon (position in, three keys out), three stable
    (key, index) sorts at 16 B per photon each (one read + one write of the 8-B pair), the 16-B records
    gathered (4 B index + 16 B gather + 16 B write per list); per top level (while nodes hold more than
    256 photons) each list's 16-B record read and written plus its 4-B segment number read; the subtree
    pass reads the three lists (48 B), writes 2n - 1 nodes (32 B per photon) and the map's records in kd
    order (position + direction + colour, 36 B)."""
    if n <= 0:
        return 0.0
    levels, m = 0, n
    while m > 256:
        m = (m + 1) // 2
        levels += 1
    return n * (28.0 + 3 * 16.0 + 3 * 36.0 + levels * 3 * 36.0 + 48.0 + 32.0 + 36.0)


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
        if a.gpus not in (1, world):
            print(f"bench: --gpus {a.gpus} under torch.distributed.run with WORLD_SIZE {world}: using {world} ranks", file=sys.stderr)
        n_gpus = world
    else:
        torch.cuda.set_device(0)
        n_gpus = max(1, a.gpus)
        if n_gpus > torch.cuda.device_count():
            raise SystemExit(f"bench: --gpus {n_gpus} but {torch.cuda.device_count()} devices are visible")

    import libyafaray_amd as Y
    from libyafaray_amd import scenes
    if a.scene == "sphere":
        spec = scenes.cornell_sphere(width=a.width, height=a.height, spp=a.spp, bounces=a.bounces, rr=not a.no_rr)
    elif a.scene == "photon":
        spec = scenes.cornell_photon(a.width, a.height, spp=a.spp, photons=a.photons)
        if a.fg:
            spec = dataclasses.replace(spec, render=dataclasses.replace(spec.render, pm_final_gather=True, fg_samples=a.fg))
    elif a.scene == "meshlight":
        spec = scenes.cornell_meshlight(a.width, a.height, spp=a.spp, bounces=a.bounces, rr=not a.no_rr, shape="bigsphere",
                                        double_sided=True, keep_area=True, samples=1)
    else:
        spec = scenes.cornell(a.width, a.height, spp=a.spp, bounces=a.bounces, rr=not a.no_rr)
    if a.lights > 1:
        spec = scenes.with_extra_lights(spec, a.lights)
    yi = Y.Interface()
    scenes.apply(spec, yi)
    yi.L.yafaray_amd_setChunkSlots(yi.h, a.chunk)
    if world > 1:
        # the library renders this rank's row band and all-gathers the bands over RCCL itself
        Y.join_render_group(yi, rank, world, dist)
    # one process: exactly n_gpus devices (the default "gpus" = -1 would take every visible GPU)
    mpg = max(1, a.members_per_gpu)
    yi.set_device_group(mpg if world > 1 else n_gpus * mpg,
                        [local_rank] * mpg if world > 1 else [d for d in range(n_gpus) for _ in range(mpg)])
    if not yi.L.yafaray_amd_buildAccelerator(yi.h):
        raise RuntimeError(yi.last_error())
    W, H = a.width, a.height

    def sync():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
            torch.cuda.synchronize()

    for _ in range(a.warmup):
        yi.render_quiet()
    # the traversal's per-visit node / triangle counters of this (deterministic) frame: one untimed
    # frame with them, the timed frames without (yafaray_amd_setTraceStats; rays are counted always)
    yi.render_quiet()
    trav = {k: yi.stats()[k] for k in ("node_visits", "tri_tests")}
    yi.L.yafaray_amd_setTraceStats(yi.h, 0)
    # timed region: every launch bracketed by HIP events on the render stream (profile mode)
    yi.L.yafaray_amd_setProfileKernels(yi.h, 1)
    sync()
    t0 = time.perf_counter()
    stats_acc, kt_acc = [], []
    for _ in range(a.steps):
        yi.render_quiet()
        stats_acc.append(yi.stats())
        kt_acc.append(yi.kernel_times())
    sync()
    elapsed = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([elapsed], device="cuda", dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t.item())
        tot = torch.tensor([sum(s["closest_rays"] + s["shadow_rays"] for s in stats_acc)], device="cuda", dtype=torch.float64)
        dist.all_reduce(tot)
        rays_total = float(tot[0].item())
    else:
        rays_total = float(sum(s["closest_rays"] + s["shadow_rays"] for s in stats_acc))

    samples_total = float(W * H * a.spp * a.steps)     # whole job: every rank's band together
    msps = samples_total / elapsed / 1e6
    mrays = rays_total / elapsed / 1e6

    # the reference's render() ends with the film's flush to the client (imagefilm.cc:570-670 via
    # scene.cc:203-263); renderQuiet keeps the normalised film on the GPU.  yafaray_render with a flush
    # callback (the film downloaded to the host, then the callback), timed beside the value's frames
    flush_ms = None
    if world <= 1 and a.flush_steps > 0:
        yi.L.yafaray_amd_setProfileKernels(yi.h, 0)
        # one untimed flushed frame first: the host film (page-locked, reused across frames) is allocated there
        yi.render(flush=lambda: None)
        sync()
        t0 = time.perf_counter()
        for _ in range(a.flush_steps):
            yi.render(flush=lambda: None)
        sync()
        flush_ms = (time.perf_counter() - t0) / a.flush_steps * 1e3

    s, kt = dict(stats_acc[-1]), kt_acc[-1]
    s.update(trav)   # node visits / triangle tests of the stats frame
    pmc = load_pmc(a, W, H)
    kernels, frame_ms = kernel_table(a, s, kt, pmc)
    roof = dominant_roofline(s, kt, kernels, pmc, a.scene)

    cpu, parity = None, None
    group = None
    grouped = n_gpus > 1 or mpg > 1
    if grouped:
        # a multi-GPU speed never goes out without its parity verdict (--no-parity does not apply):
        # the group's frame against a one-member render, and an RR-off group frame against the oracle
        # around the band boundaries (group_parity).  --members-per-gpu > 1 on one GPU rehearses the
        # same code path (logical members, one stream each) and is checked the same way
        report = yi.group_report()
        film = yi.film() if rank == 0 else None
        rr_off = scenes.cornell(W, H, spp=a.spp, bounces=a.bounces, rr=False) if a.scene == "cornell" else None
        members = n_gpus * mpg if world <= 1 else world
        devices = None if world > 1 else [d for d in range(n_gpus) for _ in range(mpg)]
        t_gp = time.perf_counter()
        parity = group_parity(Y, spec, film, report, members, devices=devices, rr_off_spec=rr_off,
                              chunk=a.chunk, world=world, rank=rank, dist=dist)
        parity["check_seconds"] = round(time.perf_counter() - t_gp, 2)
        group = report
    if rank == 0 and not grouped:
        if not a.no_cpu_baseline:
            cpu, band = cpu_baseline(spec, a)
            if not a.no_parity and band is not None:
                rgba, w = yi.film()
                parity = {"band": band_parity(spec, rgba, w, band)}
                if spec.render.rr_min_bounces < spec.render.bounces:
                    parity["band_seed2"] = second_seed_parity(Y, spec, a, band)
        if not a.no_parity and a.scene == "cornell":
            parity = parity or {}
            parity["rr_off_bitexact"] = rr_off_parity(Y, a)

    if rank == 0:
        out = {
            "metric": METRIC,
            "value": round(msps, 3),
            "unit": "Msamples/s",
            "n_gpus": n_gpus,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            # yafaray_render incl. the film's download to the host and the flush callback (not the value)
            "ms_per_step_flush": round(flush_ms, 3) if flush_ms is not None else None,
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f32",
            "data": "synthetic (Cornell box scene generated in-repo, SURVEY.md §8d)",
            "config": {"workload": workload_name(a, W, H),
                       "width": W, "height": H, "spp": a.spp, "bounces": a.bounces,
                       "samples_per_step": W * H * a.spp,
                       "parallelism": (f"row-bands x{world} (render group: one process per GPU, in-library RCCL all-gather)" if world > 1
                                       else f"row-bands x{n_gpus} (device group: one process, one thread + stream per GPU, bands pulled over xGMI)"
                                       if n_gpus > 1 else "one GPU"),
                       "chunk_slots": a.chunk},
            "mrays_per_s": round(mrays, 2),
            "rays_per_sample": round(rays_total / samples_total, 3),
            "roofline": roof,
            "kernels": kernels,
            "kernel_ms_per_step": round(frame_ms, 3),
            "photon_map": ({"photons_stored": s["photons"], "seconds_per_step": round(s["photon_seconds"], 4),
                            "shoot_seconds": round(s["photon_shoot_seconds"], 4), "tree_seconds": round(s["photon_tree_seconds"], 4),
                            **({"radiance_points": s["radiance_points"], "radiance_photons": s["radiance_photons"],
                                "fg_thin_seconds": round(s["fg_thin_seconds"], 4), "fg_radiance_seconds": round(s["fg_radiance_seconds"], 4),
                                "fg_thin_rounds": s["fg_thin_rounds"]}
                               if a.fg else {})}
                           if a.scene == "photon" else None),
            "launch": {k: s[k] for k in ("trace_grid", "shade_grid", "trace_block", "stack_depth", "scene_in_lds", "bvh_nodes")},
            # accelerator build + scene upload, once before the timed region (the reference builds
            # its kd-tree inside render(), scene.cc:218)
            "scene_build_seconds": round(s["build_seconds"], 4),
            "parity": parity,
            "cpu_baseline": cpu,
            "build": {"lib_sha256": Y.lib_sha256(), "flags": Y.build_info()},
        }
        if group is not None:
            out["group"] = {k: group.get(k) for k in ("mode", "members", "devices", "peer_devices", "peer_access", "copy_path", "bounds",
                                                      "member_ms")}
        print(json.dumps(out))
    yi.close()
    if world > 1:
        dist.destroy_process_group()
    if parity is not None and grouped and not parity.get("pass", False):
        print("bench: multi-GPU parity FAILED (see the line's parity object)", file=sys.stderr)
        sys.exit(3)


def kernel_table(a, s, kt, pmc):
    """Per kernel kind: ms per frame, share, launches, algorithmic bytes, measured traffic, fraction."""
    frame_ms = sum(v["ms"] for v in kt.values())
    in_lds = bool(s["scene_in_lds"])
    out = {}
    for kind, v in sorted(kt.items(), key=lambda kv: -kv[1]["ms"]):
        e = {"ms": round(v["ms"], 3), "share": round(v["ms"] / frame_ms, 4) if frame_ms else None, "launches": v["launches"],
             "items": v["items"]}
        ab = algo_bytes(kind, s, v, in_lds, a, kt)
        if ab is not None and v["ms"] > 0:
            e["algo_bytes_per_item"] = round(ab / max(1, v["items"]), 1)
            e["achieved_gbs"] = round(ab / (v["ms"] * 1e-3) / 1e9, 1)
            e["frac"] = round(ab / (v["ms"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)
        p = (pmc or {}).get("kernels", {}).get(kind)
        # frames the PMC pass rendered: one k_film per (single-pass) frame
        frames = ((pmc or {}).get("kernels", {}).get("k_film") or {}).get("dispatches")
        if p and "hbm_bytes_per_launch" in p and v["ms"] > 0 and v["launches"]:
            # measured per launch (the PMC pass may span several frames: its total is not one frame's); a
            # kind made of several kernels (pkd_build, photon_compact: one launch record per frame) is its
            # total over the pass's frames
            if kind not in SINGLE_KERNEL_KINDS and frames and "hbm_bytes_total" in p:
                # the pass's total over its frames = one frame's bytes of this kind, whatever the number of
                # launch records per frame (C5 + FG: two trees)
                e["traffic_bytes"] = int(p["hbm_bytes_total"] / frames)
            else:
                e["traffic_bytes"] = int(p["hbm_bytes_per_launch"] * v["launches"])
            e["traffic_gbs"] = round(e["traffic_bytes"] / (v["ms"] * 1e-3) / 1e9, 1)
            e["traffic_frac"] = round(e["traffic_gbs"] / HBM_PEAK_GBS, 4)
            if p.get("hbm_bytes_per_launch") and "write_bytes_per_launch" in p:
                # a write-only stream (k_camera) runs above the guide's 6.29 TB/s, which is a float4 copy
                e["traffic_write_frac"] = round(p["write_bytes_per_launch"] / p["hbm_bytes_per_launch"], 4)
            if "valu_lane_util" in p:
                e["valu_lane_util"] = p["valu_lane_util"]
            if "sq_insts_valu_per_launch" in p and v["launches"] and kind in SINGLE_KERNEL_KINDS:
                e["valu_issue_frac"] = round(p["sq_insts_valu_per_launch"] / (v["ms"] / v["launches"] * 1e-3) / 1e9 / VALU_PEAK_GIPS, 4)
        out[kind] = e
    return out, frame_ms


def dominant_roofline(s, kt, kernels, pmc, scene=None):
    """The contract's roofline object for the kernel with the largest share of the frame."""
    if not kt:
        return None
    kind = max(kt, key=lambda k: kt[k]["ms"])
    v, e = kt[kind], kernels[kind]
    launches = max(1, v["launches"])
    avg_ms = v["ms"] / launches
    achieved = e.get("achieved_gbs", 0.0)
    per_launch = achieved * 1e9 * avg_ms * 1e-3
    p = (pmc or {}).get("kernels", {}).get(kind, {})
    traffic = p.get("hbm_bytes_per_launch")
    if e.get("traffic_bytes") is not None:
        traffic = round(e["traffic_bytes"] / launches)   # per launch record of this kind (multi-kernel kinds: per frame)
    roof = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "kernel": kind, "avg_launch_ms": round(avg_ms, 4), "launches_per_step": launches,
            "algo_bytes_per_launch": round(per_launch)}
    if e.get("traffic_gbs") is not None:
        # the PMC-measured HBM rate of the same kernel next to the algorithmic one
        roof["traffic_gbs"] = e["traffic_gbs"]
        roof["traffic_frac"] = e["traffic_frac"]
    if kind == "k_shade":
        roof["model"] = "SURVEY §8d: 64 B of path state per segment"
        if e.get("traffic_gbs") is not None:
            roof["limiter"] = (f"HBM: {round(p['hbm_bytes_per_launch'] / max(1, v['items'] / launches))} B per vertex measured "
                               f"(the wavefront keeps path state, queues and the deferred NEE estimate in HBM between launches; "
                               f"DESIGN.md §5 byte accounting) at {e['traffic_gbs']} GB/s = {e['traffic_frac']} of peak")
    if kind == "k_trace" and scene in SURVEY_B_RAY:
        # §8d's per-ray model (the reference kd-tree's node / triangle counts) next to our BVH4 bytes
        bc, bs = SURVEY_B_RAY[scene]
        model = (bc * s["closest_rays"] + bs * s["shadow_rays"]) / launches
        rate = model / (avg_ms * 1e-3) / 1e9
        roof["survey_per_ray_model"] = {"closest_B": bc, "shadow_B": bs, "bytes_per_launch": round(model),
                                        "achieved": round(rate, 1), "frac": round(rate / HBM_PEAK_GBS, 4)}
        if not s["scene_in_lds"]:
            # the scene streams from L2 / MALL / HBM: the per-ray model is the headline (the BVH4
            # bytes of every visit, 128 B, overstate the node data a kd-tree ray would touch)
            roof["achieved"] = round(rate, 1)
            roof["frac"] = round(rate / HBM_PEAK_GBS, 4)
            roof["algo_bytes_per_launch"] = round(model)
            roof["model"] = "SURVEY §8d per-ray bytes"
        else:
            roof["model"] = "ray I/O (the LDS-resident scene's traversal bytes never reach HBM)"
    if kind == "k_trace":
        trav = NODE_BYTES.get(s["bvh_width"], 64.0) * s["node_visits"] + 48.0 * s["tri_tests"]
        rate = trav / launches / (avg_ms * 1e-3) / 1e9
        rays = max(1, s["closest_rays"] + s["shadow_rays"])
        roof["traversal"] = {"bytes_per_launch": round(trav / launches), "served_from": "LDS" if s["scene_in_lds"] else "L2/MALL/HBM",
                             "achieved": round(rate, 1), "unit": "GB/s", "lds_peak": LDS_PEAK_GBS,
                             "frac_of_lds_peak": round(rate / LDS_PEAK_GBS, 4), "bvh_width": s["bvh_width"],
                             "node_visits_per_ray": round(s["node_visits"] / rays, 2), "tri_tests_per_ray": round(s["tri_tests"] / rays, 2)}
        if "valu_issue_frac" in e:
            roof["valu"] = {"issue_frac": e["valu_issue_frac"], "lane_util": e.get("valu_lane_util")}
            if e.get("valu_lane_util") is not None:
                useful = round(e["valu_issue_frac"] * e["valu_lane_util"], 4)
                roof["valu"]["useful_frac"] = useful
                if s["scene_in_lds"]:
                    # C2: what bounds the kernel is instruction issue under divergence, not HBM
                    roof["limiter"] = (f"VALU: issue {e['valu_issue_frac']} x lane utilisation {e['valu_lane_util']} = "
                                       f"{useful} of peak useful lanes (LDS-resident scene)")
    return roof


# ---------------------------------------------------------------------------------------------
# CPU baseline + parity
# ---------------------------------------------------------------------------------------------
def host_cpu():
    """(threads, nproc, model): the threads the CPU baseline runs = the cores this job may use —
    the scheduler affinity, capped by the box's CPU share when the pool states one in
    OMP_NUM_THREADS (the GPU pool gives each one-GPU job 16 of the host's cores and shows the
    whole machine in nproc; measured: 256 threads on such a box ran slower than 16)."""
    try:
        n_aff = len(os.sched_getaffinity(0))
    except Exception:
        n_aff = os.cpu_count() or 1
    share = int(os.environ.get("OMP_NUM_THREADS", "0") or 0)
    if share > 0:
        n_aff = min(n_aff, share)
    model = platform.processor() or ""
    try:
        for line in subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout.splitlines():
            if line.startswith("Model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return n_aff, os.cpu_count() or 1, model


def cpu_baseline(spec, a):
    """The CPU oracle (C++ restatement of the reference loop, std::thread per core) on every core this
    process may run on, over a bounded band of rows of the same frame, scaled to Msamples/s.
    Returns (cpu_baseline dict, (y0, y1, rgba, weights) of the band or None)."""
    try:
        from oracle import oracle as O
    except Exception as e:  # pragma: no cover
        return {"error": str(e)}, None
    cores, nproc, model = host_cpu()
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
    # probe 4 rows, then size the band to ~cpu_seconds
    ts = spec.render.tile_size
    y0 = (spec.render.height // 2 // ts) * ts
    t0 = time.perf_counter()
    osc.render(y0, y0 + 4)
    per_row = (time.perf_counter() - t0) / 4
    rows = int(max(8, min(spec.render.height - y0, a.cpu_seconds / max(per_row, 1e-6))))
    t0 = time.perf_counter()
    rgba, w, ctr = osc.render(y0, y0 + rows)
    dt = time.perf_counter() - t0
    n = rows * spec.render.width * spec.render.aa_samples
    base = {"unit": "Msamples/s", "cores": cores, "kind": "port", "nproc": nproc, "cpu_model": model,
            "threads": cores, "threads_rule": "sched affinity capped by OMP_NUM_THREADS (the box's CPU share)"}
    band = None if spec.render.integrator == "photonmapping" else (y0, y0 + rows, rgba, w)
    if t_photons > 0.0:
        frame = spec.render.width * spec.render.height * spec.render.aa_samples
        t_frame = t_photons + dt * frame / n
        base.update({"value": round(frame / t_frame / 1e6, 4),
                     "sample": f"rows {y0}..{y0 + rows} of the {spec.render.width}x{spec.render.height} frame "
                               f"({n} samples, {dt:.1f} s, {cores} threads){photon_note}"})
        return base, band
    base.update({"value": round(n / dt / 1e6, 4), "mrays_per_s": round((ctr[0] + ctr[1]) / dt / 1e6, 3),
                 "sample": f"rows {y0}..{y0 + rows} of the same {spec.render.width}x{spec.render.height}x"
                           f"{spec.render.aa_samples}spp frame ({n} samples, {dt:.1f} s, {cores} threads)"})
    return base, band


def band_parity(spec, rgba, w, band):
    """GPU frame vs the oracle's band.  The band's first row lacks the splats of the row above it
    (forward-only footprint), so rows y0+1..y1-1 are compared.  Russian roulette on: the reference's
    RR draws are tile-order dependent, so the check is statistical — the paired
    difference image's 8x8 block means (oracle/stats.py): a frame-wide bias shows as |mean_z| >= 4,
    a local one as a block |z| >= 6; without RR it is exact."""
    from oracle.stats import paired_z
    y0, y1, orgba, ow = band
    rr = spec.render.rr_min_bounces < spec.render.bounces
    res = {"rows": [y0 + 1, y1], "pixels": int((y1 - y0 - 1) * rgba.shape[1]), "rr": rr,
           "weights_equal": bool(np.array_equal(w[y0 + 1:y1], ow[y0 + 1:y1]))}
    z = paired_z(rgba[y0 + 1:y1], orgba[y0 + 1:y1])
    res.update({"blocks": z["blocks"], "max_abs_z": round(z["max_abs_block_z"], 3),
                "frac_abs_z_gt_4": round(z["frac_abs_block_z_gt_4"], 5), "mean_z": round(z["mean_z"], 3),
                "mean_diff": z["mean_diff"], "mean_diff_se": z["mean_diff_se"], "mean_rel_diff": round(z["mean_rel_diff"], 6)})
    if not rr:
        res["bit_identical"] = bool(np.array_equal(rgba[y0 + 1:y1].view(np.uint32), orgba[y0 + 1:y1].view(np.uint32)))
    res["pass"] = bool(res["weights_equal"] and (res.get("bit_identical", True)) and res["max_abs_z"] < 6.0
                       and abs(res["mean_z"]) < 4.0)
    return res


def second_seed_parity(Y, spec, a, band, seed=7919):
    """The RR-on band check again with an independent RR seed on both sides (GPU adv_rr_seed, oracle
    rr_seed): one more GPU frame, the oracle on the same rows."""
    from libyafaray_amd import scenes
    from oracle import oracle as O
    y0, y1 = band[0], band[1]
    s2 = spec.with_render(rr_seed=seed)
    yi = Y.Interface()
    scenes.apply(s2, yi)
    yi.set_device_group(1, [0])
    yi.L.yafaray_amd_setChunkSlots(yi.h, a.chunk)
    yi.render_quiet()
    rgba, w = yi.film()
    yi.close()
    cores, _, _ = host_cpu()
    orgba, ow, _ = O.OracleScene(s2, threads=cores, rr_seed=seed).render(y0, y1)   # full-size arrays, rows y0..y1 filled
    res = band_parity(s2, rgba, w, (y0, y1, orgba, ow))
    res["rr_seed"] = seed
    return res


def _bits_equal(x, y):
    return bool(np.array_equal(np.ascontiguousarray(x, np.float32).view(np.uint32), np.ascontiguousarray(y, np.float32).view(np.uint32)))


def group_parity(Y, spec, group_film, report, members, devices=None, rr_off_spec=None, chunk=None, world=1, rank=0, dist=None,
                 rows_per_boundary=6):
    """The multi-GPU frame checked against what it must equal (imagesplitter.cc:30-107 and
    integrator_tiled.cc:246-264: the film does not depend on how many workers render it):
      (a) `group_film` (rgba, weights) — the group's frame — bit for bit against a one-member render of
          the same frame on this process's first device (the band split is bit-invariant by design:
          pixel-major RR seeds, halo rows, the one-thread splat order);
      (b) `rr_off_spec` (the same scene, Russian roulette off) rendered by a group of the same shape,
          against the CPU oracle on rows around the first and the last band boundary, bit for bit.
    `report` is the library's group report of the checked render (yafaray_amd_getGroupReport): devices,
    peer-access matrix, copy path, band bounds, per-member ms.  One process: a device group of
    `members` on `devices` (None: logical members on the current device).  torch.distributed (world > 1):
    every rank calls this; (b) renders with a fresh render group of all ranks, rank 0 compares, and the
    verdict is broadcast so every rank agrees.  Returns the parity dict (rank 0; other ranks: pass only)."""
    from libyafaray_amd import scenes
    res = {"group": report, "members": members if world <= 1 else world}
    ok = True
    # (a) one member, same frame
    if rank == 0:
        yi = Y.Interface()
        scenes.apply(spec, yi)
        dev0 = devices[0] if devices else (report.get("devices") or [0])[0]
        yi.set_device_group(1, [dev0])
        if chunk:
            yi.L.yafaray_amd_setChunkSlots(yi.h, chunk)
        t0 = time.perf_counter()
        yi.render_quiet()
        t1 = time.perf_counter() - t0
        one_rgba, one_w = yi.film()
        yi.close()
        g_rgba, g_w = group_film
        diff = np.ascontiguousarray(g_rgba, np.float32).view(np.uint32) != np.ascontiguousarray(one_rgba, np.float32).view(np.uint32)
        rows_bad = np.nonzero(diff.any(axis=(1, 2)))[0]
        res["vs_one_member"] = {"bit_identical": _bits_equal(g_rgba, one_rgba), "weights_equal": _bits_equal(g_w, one_w),
                                "rows_differing": int(len(rows_bad)), "first_bad_rows": [int(r) for r in rows_bad[:8]],
                                "one_member_frame_s": round(t1, 3)}
        ok = ok and res["vs_one_member"]["bit_identical"] and res["vs_one_member"]["weights_equal"]
    # (b) RR off on the group against the oracle, rows around the band boundaries
    if rr_off_spec is not None:
        yi = Y.Interface()
        scenes.apply(rr_off_spec, yi)
        if world > 1:
            Y.join_render_group(yi, rank, world, dist)
            yi.set_device_group(1, [(report.get("devices") or [0])[0]])
        else:
            yi.set_device_group(members, devices)
        if chunk:
            yi.L.yafaray_amd_setChunkSlots(yi.h, chunk)
        yi.render_quiet()
        rep = yi.group_report()
        if rank == 0:
            rgba, w = yi.film()
        yi.close()
        if rank == 0:
            from oracle import oracle as O
            H = rr_off_spec.render.height
            b = rep["bounds"] or [0, H]
            inner = b[1:-1] or [H // 2]
            picks = sorted({inner[0], inner[-1]})
            cores, _, _ = host_cpu()
            osc = O.OracleScene(rr_off_spec, threads=cores)
            checks = []
            t0 = time.perf_counter()
            for yb in picks:
                y0, y1 = max(0, yb - rows_per_boundary // 2 - 1), min(H, yb + rows_per_boundary // 2)
                orgba, ow, _ = osc.render(y0, y1)
                a_ = rgba[y0 + 1:y1].view(np.uint32).astype(np.int64)
                o_ = orgba[y0 + 1:y1].view(np.uint32).astype(np.int64)
                checks.append({"boundary": int(yb), "rows": [y0 + 1, y1], "bit_identical": bool(np.array_equal(a_, o_)),
                               "max_ulp": int(np.abs(a_ - o_).max()) if a_.size else 0,
                               "weights_equal": bool(np.array_equal(w[y0 + 1:y1], ow[y0 + 1:y1]))})
            res["rr_off_vs_oracle"] = {"bounds": b, "checks": checks, "cpu_s": round(time.perf_counter() - t0, 2)}
            ok = ok and all(c["bit_identical"] and c["weights_equal"] for c in checks)
    if world > 1 and dist is not None:
        import torch
        t = torch.tensor([1 if ok else 0], device="cuda", dtype=torch.int32)
        dist.broadcast(t, src=0)
        ok = bool(t.item())
    res["pass"] = bool(ok)
    return res


def rr_off_parity(Y, a):
    """The same full-size frame with Russian roulette off, rendered on the GPU, against the oracle
    on a band of rows: bit for bit (the reference's integrator without RR is deterministic)."""
    from libyafaray_amd import scenes
    from oracle import oracle as O
    spec = scenes.cornell(a.width, a.height, spp=a.spp, bounces=a.bounces, rr=False)
    yi = Y.Interface()
    scenes.apply(spec, yi)
    yi.set_device_group(1, [0])
    yi.L.yafaray_amd_setChunkSlots(yi.h, a.chunk)
    t0 = time.perf_counter()
    yi.render_quiet()
    t_gpu = time.perf_counter() - t0
    rgba, w = yi.film()
    yi.close()
    cores, _, _ = host_cpu()
    y0 = a.height // 3
    y1 = min(a.height, y0 + max(2, a.parity_rows))
    t0 = time.perf_counter()
    orgba, ow, _ = O.OracleScene(spec, threads=cores).render(y0, y1)
    t_cpu = time.perf_counter() - t0
    a_ = rgba[y0 + 1:y1].view(np.uint32)
    b_ = orgba[y0 + 1:y1].view(np.uint32)
    ulp = np.abs(a_.astype(np.int64) - b_.astype(np.int64))
    return {"rows": [y0 + 1, y1], "pixels": int(a_.shape[0] * a_.shape[1]), "bit_identical": bool(np.array_equal(a_, b_)),
            "max_ulp": int(ulp.max()), "weights_equal": bool(np.array_equal(w[y0 + 1:y1], ow[y0 + 1:y1])),
            "gpu_frame_s": round(t_gpu, 3), "cpu_band_s": round(t_cpu, 2)}


if __name__ == "__main__":
    main()
