"""Host enqueue time vs GPU time of the training step (development tool): for a window of steps after W
warm-up steps, the time neus_testbed_train takes to return (host enqueue) and the time until the stream
drains, plus the per-phase GPU times from the testbed's phase events."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from neus2_amd import pyngp, scenes
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
done = 0
for w, n in ((5, 20), (200, 20), (800, 20)):
    tb.train_steps(w - done); tb.synchronize(); done = w
    t0 = time.perf_counter(); tb.train_steps(n); t1 = time.perf_counter(); tb.synchronize(); t2 = time.perf_counter()
    done += n
    tb.set_profiling(True); tb.train_steps(n); tb.synchronize(); done += n
    ph = tb.phase_times(); tb.set_profiling(False)
    st = tb.stats()
    print(f"   march first pass {st['march_first_pass_rays']} kept extent {st['kept_ray_extent']} Npre {st['measured_batch_size_before_compaction']}", flush=True)
    print(f"after {w}: enqueue {1e3 * (t1 - t0) / n:.3f} ms/step, wall {1e3 * (t2 - t0) / n:.3f} ms/step, phases {ph}", flush=True)
