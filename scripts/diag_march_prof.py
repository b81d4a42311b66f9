"""Phase timing of the occupancy march's first pass on the bench workload (development tool): per wave, wall-clock
stamps at start / slice start reached / segment marched / joined / counted / written (neus_debug_march_profile)."""
import ctypes as C
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
from neus2_amd import pyngp, scenes  # noqa: E402
from neus2_amd._lib import check, lib  # noqa: E402

torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
tb.train_steps(int(os.environ.get("WARM", "800")))
tb.synchronize()
nw = (1 << 18) * 8 // 64
buf = np.zeros(nw * 8, np.uint64)
n = C.c_uint32()
for rep in range(3):
    check(lib().neus_debug_march_profile(tb.handle, buf.ctypes.data_as(C.POINTER(C.c_ulonglong)), nw, C.byref(n)))
p = buf.reshape(-1, 8).astype(np.int64)
act = p[:, 0] > 0
q = p[act]
t0 = q[:, 0].min()
st, en = (q[:, 0] - t0) / 100.0, (q[:, 5] - t0) / 100.0  # us
ph = np.diff(q[:, :6], axis=1) / 100.0
samples, redo = q[:, 6], q[:, 7] & 0xff
ev_max, ev_sum = q[:, 7] >> 32, (q[:, 7] >> 8) & 0xffffff
print(f"waves with stamps {act.sum()} of {nw}; kernel span {en.max():.1f} us (first start .. last end)")
print(f"wave start: p50 {np.median(st):.1f} p99 {np.percentile(st, 99):.1f} max {st.max():.1f} us")
print(f"wave duration: mean {(en - st).mean():.1f} p50 {np.median(en - st):.1f} p99 {np.percentile(en - st, 99):.1f} max {(en - st).max():.1f} us")
names = ["slice start", "segment march", "join", "count", "write"]
for k, nm in enumerate(names):
    print(f"  {nm:14s} mean {ph[:, k].mean():7.2f} p50 {np.median(ph[:, k]):7.2f} p99 {np.percentile(ph[:, k], 99):7.2f} max {ph[:, k].max():7.2f} us")
busy = samples > 0
print(f"waves with samples {busy.sum()}; samples per such wave mean {samples[busy].mean():.0f} max {samples.max()}; redo rounds mean {redo.mean():.2f} max {redo.max()}")
print(f"segment events per wave: lane max mean {ev_max[busy].mean():.1f} p99 {np.percentile(ev_max[busy], 99):.0f}; lane mean {(ev_sum[busy] / 64).mean():.1f}; "
      f"segment-march us per max-lane event {np.median(ph[busy, 1] / np.maximum(ev_max[busy], 1)):.3f}")
crit = np.argmax(en)
print(f"critical wave: start {st[crit]:.1f} dur {en[crit] - st[crit]:.1f} phases {np.round(ph[crit], 1).tolist()} samples {samples[crit]} redo {redo[crit]} events max {ev_max[crit]}")
order = np.argsort(-(en - st))[:10]
for i in order:
    print(f"   long wave: start {st[i]:7.1f} dur {en[i] - st[i]:7.1f} phases {np.round(ph[i], 1).tolist()} samples {samples[i]} redo {redo[i]} events max {ev_max[i]} sum {ev_sum[i]}")
# concurrency over time: waves running at t
ts = np.linspace(0, en.max(), 20)
print("running waves over time:", [int(((st <= t) & (en > t)).sum()) for t in ts])
