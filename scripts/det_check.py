import os, sys
sys.path.insert(0, '/root/repo'); sys.path.insert(0, '/root/repo/tests')
import numpy as np, torch
torch.cuda.set_device(0)
from neus2_amd import pyngp, scenes
sc = scenes.small_scene(n_views=8, width=64, height=48)
ROOT='/root/repo'
def mk(mode):
    if mode: os.environ['NEUS_SCATTER'] = mode
    else: os.environ.pop('NEUS_SCATTER', None)
    tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
    tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
    tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=4096)
    os.environ.pop('NEUS_SCATTER', None)
    return tb
res = {}
for name, mode in [('r1', None), ('r2', None), ('b1', 'binned'), ('b2', 'binned')]:
    tb = mk(mode)
    ps = []
    for k in range(40):
        tb.train_steps(1)
        ps.append(tb.get_params().copy())
    res[name] = ps
def first_diff(a, b):
    for k in range(40):
        if not np.array_equal(a[k].view(np.uint32), b[k].view(np.uint32)):
            d = np.nonzero(a[k].view(np.uint32) != b[k].view(np.uint32))[0]
            return k, len(d), d[:5]
    return None
print('r1 vs r2', first_diff(res['r1'], res['r2']))
print('b1 vs b2', first_diff(res['b1'], res['b2']))
print('r1 vs b1', first_diff(res['r1'], res['b1']))
