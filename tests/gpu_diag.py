"""Diagnostics for a GPU box run: ULP histograms GPU vs oracle and small timings."""
import sys, os, time, json
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import libyafaray_amd as Y
from libyafaray_amd import scenes
from oracle import oracle as O

def ulp(a, b):
    a = np.ascontiguousarray(a, np.float32).view(np.int32).astype(np.int64)
    b = np.ascontiguousarray(b, np.float32).view(np.int32).astype(np.int64)
    return np.abs(a - b)

for name, spec, chunk in [
    ("test01 DL 128x128x4", scenes.test01(128, 128, spp=4), None),
    ("cornell PT noRR 160x90x16", scenes.cornell(160, 90, spp=16, rr=False), 65536),
    ("cornell PT RR 160x90x16", scenes.cornell(160, 90, spp=16, rr=True), 65536),
    ("cornell DL 160x90x4 gauss", scenes.cornell(160, 90, spp=4, integrator="directlighting", filter_type="gauss", pixelwidth=1.5), None),
]:
    t = time.time(); g, gw, st = Y.render_spec(spec, chunk_slots=chunk); tg = time.time() - t
    t = time.time(); o, ow, oc = O.OracleScene(spec, threads=16).render(); to = time.time() - t
    d = ulp(g, o)
    print(f"{name}: gpu {tg:.2f}s oracle {to:.2f}s | equal {np.mean(d == 0)*100:.3f}% max_ulp {d.max()} | mean g {g[...,:3].mean():.6f} o {o[...,:3].mean():.6f} | rays gpu {st['closest_rays']}+{st['shadow_rays']} oracle {oc[0]}+{oc[1]} | weights equal {np.array_equal(gw, ow)}")
    print("   stats", json.dumps(st))
