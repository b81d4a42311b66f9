"""Trains WARM steps of the bench workload (Config S, base.json, R = Nc = 2^18), then STEPS more steps: the launches of
those last steps are the training step's own kernels at the bench state (development tool; run under rocprofv3 --pmc
and keep each kernel's last STEPS x launches-per-step dispatches, scripts/pmc_table.py --last)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch
from neus2_amd import pyngp, scenes
torch.cuda.set_device(0)
sc = scenes.sphere_scene(49, 1600, 1200, principal=(823.2 / 1600, 619.1 / 1200))
tb = pyngp.Testbed(pyngp.TestbedMode.Nerf)
tb.set_dataset(sc["images"], sc["focal"], sc["principal"], sc["xforms"], 1)
tb.reload_network_from_file(os.path.join(ROOT, "configs", "nerf", "base.json"), batch_size=1 << 18, fixed_rays_per_batch=1 << 18)
tb.train_steps(int(os.environ.get("WARM", "800")))
tb.synchronize()
s0 = tb.stats()
tb.train_steps(int(os.environ.get("STEPS", "5")))
tb.synchronize()
s1 = tb.stats()
print(f"steps {s1['training_step'] - s0['training_step']} progressive {s1['progressive_steps'] - s0['progressive_steps']} "
      f"evaluated {s1['evaluated_samples_total'] - s0['evaluated_samples_total']} kept {s1['pre_samples_total'] - s0['pre_samples_total']}", flush=True)
