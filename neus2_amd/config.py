"""configs/nerf/*.json surface: JSON with // comments and "parent" merging (testbed.cu:73-91,
139-162), reduced to the NeusNetworkConfig the gfx950 Testbed consumes (testbed.cu:2084-2197)."""
from __future__ import annotations

import json
import os
import re

from ._lib import NeusNetworkConfig


def _strip_comments(text: str) -> str:
    out, i, n, in_str = [], 0, len(text), False
    while i < n:
        c = text[i]
        if in_str:
            out.append(c)
            if c == "\\" and i + 1 < n:
                out.append(text[i + 1]); i += 2; continue
            if c == '"':
                in_str = False
            i += 1
            continue
        if c == '"':
            in_str = True; out.append(c); i += 1; continue
        if text.startswith("//", i):
            j = text.find("\n", i)
            i = n if j < 0 else j
            continue
        if text.startswith("/*", i):
            j = text.find("*/", i + 2)
            i = n if j < 0 else j + 2
            continue
        out.append(c); i += 1
    return "".join(out)


def _merge(parent: dict, child: dict) -> dict:
    res = dict(parent)
    for k, v in child.items():
        if isinstance(v, dict) and isinstance(res.get(k), dict):
            res[k] = _merge(res[k], v)
        else:
            res[k] = v
    return res


def load_json(path: str) -> dict:
    """Testbed::merge_parent_network_config semantics: "parent" is loaded relative to the file."""
    with open(path) as f:
        cfg = json.loads(_strip_comments(f.read()))
    if "parent" in cfg:
        parent = load_json(os.path.join(os.path.dirname(path), cfg["parent"]))
        cfg = _merge(parent, {k: v for k, v in cfg.items() if k != "parent"})
    return cfg


def parse_json_text(text: str) -> dict:
    return json.loads(_strip_comments(text))


def _leaf_optimizer(opt: dict) -> dict:
    while "nested" in opt:
        opt = opt["nested"]
    return opt


def _find(opt: dict, otype: str) -> dict:
    while True:
        if opt.get("otype", "").lower() == otype.lower():
            return opt
        if "nested" not in opt:
            return {}
        opt = opt["nested"]


def network_config(cfg: dict, batch_size: int | None = None, fixed_rays_per_batch: int = 0) -> NeusNetworkConfig:
    enc = cfg.get("encoding", {})
    net = cfg.get("network", {})
    rgb = cfg.get("rgb_network", {})
    hp = cfg.get("hyperparams", {})
    opt = cfg.get("optimizer", {})
    adam = _leaf_optimizer(opt)
    ema = _find(opt, "Ema")
    decay = _find(opt, "ExponentialDecay")
    nf = int(enc.get("n_features_per_level", 2))
    n_levels = int(enc["n_features"]) // nf if enc.get("n_features", 0) > 0 else int(enc.get("n_levels", 16))
    log2 = int(enc.get("log2_hashmap_size", 15))
    base = int(enc.get("base_resolution", 0)) or (1 << (log2 // 3))
    c = NeusNetworkConfig()
    c.n_levels = n_levels
    c.n_features_per_level = nf
    c.log2_hashmap_size = log2
    c.base_resolution = base
    c.per_level_scale = float(enc.get("per_level_scale", 0.0))
    c.top_resolution = float(enc.get("top_resolution", 2048.0))
    c.valid_level_scale = float(enc.get("valid_level_scale", 0.02))
    c.base_valid_level_scale = float(enc.get("base_valid_level_scale", 0.2))
    c.base_training_step = int(enc.get("base_training_step", 100))
    c.n_neurons = int(net.get("n_neurons", 64))
    if int(rgb.get("n_neurons", c.n_neurons)) != c.n_neurons:
        raise ValueError("density and rgb networks must share n_neurons on the gfx950 path")
    c.n_density_hidden = int(net.get("n_hidden_layers", 1))
    c.n_rgb_hidden = int(rgb.get("n_hidden_layers", 2))
    c.learning_rate = float(adam.get("learning_rate", 1e-3))
    c.beta1 = float(adam.get("beta1", 0.9))
    c.beta2 = float(adam.get("beta2", 0.999))
    c.epsilon = float(adam.get("epsilon", 1e-8))
    c.l2_reg = float(adam.get("l2_reg", 1e-8))
    c.ema_decay = float(ema.get("decay", 0.99)) if ema else 0.0
    c.decay_start = int(decay.get("decay_start", 1 << 30)) if decay else (1 << 30)
    c.decay_interval = int(decay.get("decay_interval", 10000)) if decay else 10000
    c.decay_base = float(decay.get("decay_base", 0.33)) if decay else 1.0
    c.ek_loss_weight = float(hp.get("ek_loss_weight", 0.01))
    c.mask_loss_weight = float(hp.get("mask_loss_weight", 0.0))
    c.anneal_end = int(hp.get("anneal_end", 0))
    c.batch_size = int(batch_size if batch_size is not None else hp.get("batch_size", 1 << 18))
    c.sdf_bias = -0.1
    c.density_grid_decay = 0.95
    c.seed = 1337
    c.fixed_rays_per_batch = int(fixed_rays_per_batch)
    # dynamic scenes (testbed.cu:2115-2133, 2319-2329): hyperparams + the "globalmove" optimizer (defaults: the
    # main optimizer config, as the reference falls back to it)
    c.predict_global_movement = int(bool(hp.get("predict_global_movement", False)))
    c.global_movement_steps = int(hp.get("predict_global_movement_training_step", 300))
    c.finetune_global_movement = int(bool(hp.get("finetune_global_movement", True)))
    c.reset_density_grid_after_global_movement = int(bool(hp.get("reset_density_grid_after_global_movement", True)))
    c.after_learning_rate = float(adam.get("after_learning_rate", c.learning_rate))
    gm_opt = cfg.get("globalmove", {}).get("optimizer", opt)
    gm_adam, gm_decay = _leaf_optimizer(gm_opt), _find(gm_opt, "ExponentialDecay")
    c.gm_learning_rate = float(gm_adam.get("learning_rate", 1e-3))
    c.gm_beta1 = float(gm_adam.get("beta1", 0.9))
    c.gm_beta2 = float(gm_adam.get("beta2", 0.999))
    c.gm_epsilon = float(gm_adam.get("epsilon", 1e-8))
    c.gm_decay_start = int(gm_decay.get("decay_start", 1 << 30)) if gm_decay else (1 << 30)
    c.gm_decay_interval = int(gm_decay.get("decay_interval", 10000)) if gm_decay else 10000
    c.gm_decay_base = float(gm_decay.get("decay_base", 0.33)) if gm_decay else 1.0
    if cfg.get("loss", {}).get("otype", "Huber") != "Huber":
        raise ValueError("only the Huber loss of configs/nerf/base.json is implemented on the gfx950 path")
    return c


def density_input_width(n_levels: int) -> int:
    return ((3 + 2 * n_levels) + 15) // 16 * 16
