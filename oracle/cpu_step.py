"""CPU restatement of one Testbed::train step (testbed.cu:2640-2736, testbed_nerf.cu:3440-4001) composed
from the oracle kernels — TEST INFRASTRUCTURE / CPU BASELINE ONLY (tests/, bench.py cpu_baseline).

Supports data-parallel sharding semantics (rank/world: global ray index offset rank*R, loss scale over
world*R, eikonal over world*Nc) so the gloo tests can check the N>1 decomposition on the CPU.
"""
from __future__ import annotations

import numpy as np

import oracle as O

NERF_GRID = 128


class CpuTrainer:
    def __init__(self, cfg, ds, params, batch=4096, rays_per_batch=4096, fixed_rays=False, rank=0, world=1, seed=1337):
        self.cfg, self.ds = cfg, ds
        self.lay = O.layout(cfg)
        self.params = np.ascontiguousarray(params, np.float32).copy()
        P = self.params.size
        self.m1 = np.zeros(P, np.float32)
        self.m2 = np.zeros(P, np.float32)
        self.steps = np.zeros(P, np.uint32)
        self.ema_tmp = np.zeros(P, np.float32)
        self.ema_out = np.zeros(P, np.float32)
        self.batch = batch
        self.R = rays_per_batch
        self.fixed_rays = fixed_rays
        self.rank, self.world = rank, world
        self.max_samples = batch * 16
        self.max_inference = self.max_samples
        self.n_rays_total = 0
        self.training_step = 0
        self.adam_step = 0
        # m_rng = pcg32{seed}; density_grid_rng = pcg32{m_rng.next_uint()}; tv_loss_rng (testbed.cu:2087-2101)
        r = O.pcg32(seed, 1, 0, 2)
        self.rng_state, self.rng_inc = _pcg_state(seed, 1, 2)
        self.dg_state, self.dg_inc = _pcg_state(int(r[0]), 1, 0)
        self.density_grid = np.zeros(NERF_GRID ** 3, np.float32)
        self.bitfield = np.zeros(NERF_GRID ** 3 // 8 * 8, np.uint8)  # NERF_CASCADES levels
        self.ema_step = 0
        self.last = {}

    def valid_level(self, step):
        c = self.cfg
        if step <= 0:
            return c.n_levels
        v = np.ceil(np.float32(0.2) * np.float32(c.n_levels) + np.float32(0.02) * np.float32(max(0, step - 100)))
        return int(min(c.n_levels, int(v)))

    def occupancy(self):
        step = self.training_step
        G3 = NERF_GRID ** 3
        if step == 0:
            self.density_grid[:] = 0
            self.ema_step = 0
        nu, nn = (G3, 0) if step < 256 else (G3 // 4, G3 // 4)
        self.dg_state, mean = O.density_grid_update(self.cfg, self.params, self.valid_level(step), nu, nn, self.ema_step,
                                                    self.dg_state, self.dg_inc, self.density_grid, self.bitfield)
        self.ema_step += 1
        return mean

    def march(self, skip_occupancy=False):
        """The step's occupancy update (at the reference cadence) and generate_training_samples_nerf: the rays, per-ray
        sample counts and NerfCoordinates the network then evaluates (no network arithmetic: independent of the sum order)."""
        step = self.training_step
        n_prep = min(16, max(1, step // 16))
        if not skip_occupancy and step % n_prep == 0:
            self.occupancy()
        if step == 0:
            self.n_rays_total = 0
        R, W = self.R, self.world
        rays, ns, co, counter, nr = O.generate_samples(self.ds, self.bitfield, R, self.n_rays_total, self.rng_state, self.rng_inc,
                                                       self.max_inference, ray_offset=self.rank * R, n_rays_global=W * R)
        return dict(rays=rays, numsteps=ns, coords=co, counter=counter, n_rays_with_samples=nr)

    def grads_from_march(self, m):
        """Network forward over every kept sample, the NeuS loss / compaction, the rollover and the network backward for
        the samples `march` produced; returns fp32 gradients."""
        vl = self.valid_level(self.training_step)
        R, W = self.R, self.world
        rays, ns, co = m["rays"], m["numsteps"], m["coords"]
        nk = int(ns[:, 0].sum())
        net = O.network_forward(self.cfg, self.params, co[:nk], vl)
        full = np.zeros((max(nk, 1), 16), np.uint16)
        full[:nk] = net
        res = O.compute_loss(self.ds, R, self.n_rays_total, self.rng_state, self.rng_inc, self.batch, rays, ns, co, full,
                             ray_offset=self.rank * R, n_rays_global=W * R)
        ncomp = min(res["counter"], self.batch)
        coords_c, dout = res["coords"], res["dL_dout"]
        O.fill_rollover(self.batch, ncomp, coords_c, dout)
        g = O.network_backward(self.cfg, self.params, coords_c, vl, dout, self.batch * W) if ncomp > 0 else np.zeros_like(self.params)
        self.last = dict(numsteps_counter=m["counter"], compacted=res["counter"], n_kept=nk, n_rays_with_samples=m["n_rays_with_samples"],
                         loss=float(res["loss"].sum()), rays=rays, numsteps=ns, coords=co[:nk], compacted_coords=coords_c[:ncomp],
                         dL_dout=dout[:ncomp], ray_ncomp=res["numsteps"][:, 0])
        return g

    def grads(self, skip_occupancy=False):
        """Everything of one step up to (not including) the optimizer; returns fp32 gradients."""
        return self.grads_from_march(self.march(skip_occupancy))

    def grads_alt_orders(self, m, orders=("reversed", "pairwise", "blocked")):
        """The same step's gradients with the network's layer products summed in each alternative order (the oracle's own
        spread: the noise floor of the fp16 network). self.last is left as the index-order step set it."""
        last, out = self.last, {}
        try:
            for o in orders:
                O.set_sum_order(o)
                out[o] = self.grads_from_march(m)
        finally:
            O.set_sum_order("index")
            self.last = last
        return out

    def grads_grid_mode(self, m, mode="ref_operand"):
        """The same step's gradients with the hash-grid gradient summed under another semantics (oracle.set_grid_grad_mode:
        "ref_operand" = each corner contribution rounded to fp16 as the reference's atomicAdd(__half2) operand,
        grid.h:418-421). self.last is left as the exact step set it."""
        last = self.last
        try:
            O.set_grid_grad_mode(mode)
            return self.grads_from_march(m)
        finally:
            O.set_grid_grad_mode("exact")
            self.last = last

    def finish(self, g, counters_sum=None):
        """Counters update (testbed_nerf.cu:3399-3438), RNG advance and the Ema(Adam) step."""
        W = self.world
        _, compacted = counters_sum if counters_sum is not None else (self.last["numsteps_counter"], self.last["compacted"])
        self.n_rays_total += self.R * W
        # the cap on the next step's pre-compaction samples follows this rank's own request count; the R
        # adaptation follows the all-reduced compacted count (identical on every rank)
        before, measured = self.last["numsteps_counter"], compacted // W
        if before > 0 and measured > 0:
            self.max_inference = (min(before, self.max_samples) + 127) // 128 * 128
            if not self.fixed_rays:
                r = int(np.float32(self.R) * np.float32(self.batch) / np.float32(measured))
                self.R = min((r + 127) // 128 * 128, 1 << 18)
        self.rng_state = _advance(self.rng_state, self.rng_inc, 1 << 32)
        self.adam_step += 1
        O.adam_ema_step(self.params, g, self.m1, self.m2, self.steps, self.ema_tmp, self.ema_out, self.lay["n_matrix"],
                        self.adam_step, lr=1e-3, beta1=0.9, beta2=0.99, eps=1e-15, l2=1e-6)
        self.training_step += 1

    def step(self):
        g = self.grads()
        self.finish(g)
        return g


MULT = 0x5851F42D4C957F2D
MASK = (1 << 64) - 1


def _pcg_state(initstate, initseq, n_draws):
    inc = ((initseq << 1) | 1) & MASK
    state = 0
    state = (state * MULT + inc) & MASK
    state = (state + initstate) & MASK
    state = (state * MULT + inc) & MASK
    for _ in range(n_draws):
        state = (state * MULT + inc) & MASK
    return state, inc


def _advance(state, inc, delta):
    cur_mult, cur_plus, acc_mult, acc_plus = MULT, inc, 1, 0
    while delta > 0:
        if delta & 1:
            acc_mult = (acc_mult * cur_mult) & MASK
            acc_plus = (acc_plus * cur_mult + cur_plus) & MASK
        cur_plus = ((cur_mult + 1) * cur_plus) & MASK
        cur_mult = (cur_mult * cur_mult) & MASK
        delta //= 2
    return (acc_mult * state + acc_plus) & MASK
