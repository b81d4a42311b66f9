"""Development check: two testbeds (region scatter / binned scatter) trained concurrently on their own streams,
repeated, parameters compared bitwise; prints the first differing parameter ranges of any mismatch."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np, torch
torch.cuda.set_device(0)
from neus2_amd import pyngp, scenes
sc = scenes.small_scene(n_views=8, width=64, height=48)
def mk(mode, batch):
    if mode: os.environ['NEUS_SCATTER'] = mode
    else: os.environ.pop('NEUS_SCATTER', None)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=batch)
    os.environ.pop('NEUS_SCATTER', None)
    return tb
reps = int(os.environ.get("REPS", "6"))
steps = int(os.environ.get("STEPS", "40"))
bad = 0
for rep in range(reps):
    a, b = mk(None, 4096), mk('binned' if os.environ.get("AB", "1") == "1" else None, 4096)
    a.train_steps(steps); b.train_steps(steps)
    pa, pb = a.get_params(), b.get_params()
    d = np.nonzero(pa.view(np.uint32) != pb.view(np.uint32))[0]
    lay = a.layout()
    if len(d):
        bad += 1
        print(f"rep {rep}: {len(d)} differ; first {d[:8]}; grid_offset {lay['grid_offset']} var {lay['variance_offset']}; "
              f"in MLP {int((d < lay['grid_offset']).sum())}", flush=True)
    else:
        print(f"rep {rep}: equal", flush=True)
    del a, b
print("mismatching reps", bad)
