"""GPU box: per-frame wall time of renderQuiet vs yafaray_render (flush callback) for an 8-member device group
on one GPU (C2 scene) — where does the group's flushed frame spend its time?"""
import sys, time, os
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch
import libyafaray_amd as Y
from libyafaray_amd import scenes
members = int(sys.argv[1]) if len(sys.argv) > 1 else 8
spec = scenes.cornell(1920, 1080, spp=64)
yi = Y.Interface()
scenes.apply(spec, yi)
yi.set_device_group(members, [0] * members)
yi.L.yafaray_amd_buildAccelerator(yi.h)
def t(f):
    torch.cuda.synchronize(); t0 = time.perf_counter(); f(); torch.cuda.synchronize(); return (time.perf_counter() - t0) * 1e3
for i in range(3):
    print("quiet", round(t(lambda: yi.L.yafaray_amd_renderQuiet(yi.h)), 1), flush=True)
for i in range(4):
    print("flush", round(t(lambda: yi.render(flush=lambda: None)), 1), flush=True)
for i in range(2):
    print("quiet", round(t(lambda: yi.L.yafaray_amd_renderQuiet(yi.h)), 1), flush=True)
for i in range(2):
    print("render-no-cb", round(t(lambda: yi.render()), 1), flush=True)
