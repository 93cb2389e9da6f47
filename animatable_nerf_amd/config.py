"""yacs-compatible configuration for the hot path (lib/config/config.py:9-194, lib/config/yacs.py).

Accepts the reference's yaml files (``parent_cfg`` inheritance, unknown keys kept) and CLI
``key value`` pairs, so ``--cfg_file configs/aninerf_s9p.yaml exp_name x resume False`` means the
same thing here. Only the keys the render/train path reads have typed defaults; the rest are
carried through untouched.
"""
import ast
import copy
import os

import yaml


class CfgNode(dict):
    """dict with attribute access (the subset of yacs.CfgNode the hot path uses)."""

    def __init__(self, init=None):
        super().__init__()
        for k, v in (init or {}).items():
            self[k] = CfgNode(v) if isinstance(v, dict) and not isinstance(v, CfgNode) else v

    def __getattr__(self, name):
        try:
            return self[name]
        except KeyError as e:
            raise AttributeError(name) from e

    def __setattr__(self, name, value):
        self[name] = value

    def merge(self, other):
        for k, v in other.items():
            if isinstance(v, dict):
                if not isinstance(self.get(k), CfgNode):
                    self[k] = CfgNode()
                self[k].merge(v)
            else:
                self[k] = v
        return self

    def merge_from_list(self, opts):
        """``key value`` pairs, dotted keys allowed (yacs.py:190-217); values parsed as literals."""
        if len(opts) % 2:
            raise ValueError(f'override list has odd length: {opts}')
        for k, v in zip(opts[0::2], opts[1::2]):
            node = self
            parts = k.split('.')
            for p in parts[:-1]:
                node = node.setdefault(p, CfgNode())
            node[parts[-1]] = _literal(v)
        return self

    def clone(self):
        return copy.deepcopy(self)


def _literal(v):
    if not isinstance(v, str):
        return v
    try:
        return ast.literal_eval(v)
    except (ValueError, SyntaxError):
        return v


def defaults():
    """Defaults of the keys the hot path reads (config.py:9-137 + configs/aninerf_s9p.yaml)."""
    return CfgNode({
        'task': 'deform', 'exp_name': 'hello', 'gpus': [0], 'distributed': False, 'local_rank': 0,
        'num_train_frame': 260, 'num_eval_frame': 133, 'num_latent_code': -1,
        'N_samples': 64, 'N_rand': 1024, 'perturb': 1, 'white_bkgd': False,
        'xyz_res': 10, 'view_res': 4, 'norm_th': 0.05, 'train_th': 0.0, 'box_padding': 0.05,
        'aninerf_animation': False, 'test_novel_pose': False, 'eval': False, 'train_precision': 'fp32', 'render_precision': 'fp32',
        'sdf_train_precision': 'fp32',
        'chunk': 2048, 'mesh_th': 50.0, 'voxel_size': [0.005, 0.005, 0.005],
        'train': {'lr': 5e-4, 'weight_decay': 0.0, 'optim': 'adam', 'epoch': 400,
                  'scheduler': {'type': 'exponential', 'gamma': 0.1, 'decay_epochs': 1000}},
        'ep_iter': 500, 'save_ep': 200, 'save_latest_ep': 5, 'eval_ep': 1000,
        'trained_model_dir': 'data/trained_model', 'record_dir': 'data/record', 'result_dir': 'data/result',
        'network_module': 'animatable_nerf_amd.network', 'renderer_module': 'animatable_nerf_amd.renderer',
    })


# The keys of each named experiment that reach the hot path (the yaml files are not shipped: the
# reference tree is not available where the GPU tests run). Each overrides defaults() (= aninerf_s9p).
SUBJECTS = {
    # configs/aninerf_s9p.yaml:57-93 (the defaults above); H x W 1002 x 1000 at ratio 1
    'aninerf_s9p': {'num_train_frame': 260, 'num_eval_frame': 133, 'H': 1002, 'W': 1000, 'ratio': 1.0},
    # configs/aninerf_313.yaml:23-28 (parent aninerf_s9p): ZJU-MoCap 313, 1024 x 1024 at ratio 0.5 = 512 x 512,
    # 60 training frames (nf_latent (60,128), bw_latent (61,128))
    'aninerf_313': {'num_train_frame': 60, 'num_eval_frame': 1000, 'H': 1024, 'W': 1024, 'ratio': 0.5},
    # configs/sdf_pdf/anisdf_pdf_s9p.yaml:79-95
    'anisdf_pdf_s9p': {'num_train_frame': 260, 'num_eval_frame': 133, 'H': 1002, 'W': 1000, 'ratio': 1.0,
                       'tpose_viewdir': True, 'use_bigpose': True},
}


def subject(name, **overrides):
    """defaults() with the hot-path keys of the named reference experiment (SUBJECTS) and overrides."""
    cfg = defaults()
    cfg.merge(CfgNode(SUBJECTS[name]))
    cfg.merge(CfgNode(overrides))
    if 'num_latent_code' not in overrides:
        cfg.num_latent_code = cfg.num_train_frame  # config.py:144-145
    return cfg


def load_cfg(cfg_file=None, opts=(), base_dir=None):
    """Load ``cfg_file`` (resolving ``parent_cfg`` relative to ``base_dir``) over the defaults."""
    cfg = defaults()
    if cfg_file:
        chain = []
        path = cfg_file
        while path:
            full = path if os.path.isabs(path) or base_dir is None else os.path.join(base_dir, path)
            with open(full) as f:
                node = yaml.safe_load(f) or {}
            chain.append(node)
            path = node.get('parent_cfg')
            if path and not os.path.exists(path if base_dir is None else os.path.join(base_dir, path)):
                break
        for node in reversed(chain):
            node = {k: v for k, v in node.items() if k != 'parent_cfg'}
            cfg.merge(CfgNode(node))
    cfg.merge_from_list(list(opts))
    for sub in ('aninerf_animation', 'vis_pose_sequence', 'vis_novel_view', 'vis_tpose_mesh', 'vis_posed_mesh'):
        key = {'aninerf_animation': 'aninerf_animation_cfg', 'vis_pose_sequence': 'pose_sequence_cfg',
               'vis_novel_view': 'novel_view_cfg', 'vis_tpose_mesh': 'mesh_cfg',
               'vis_posed_mesh': 'mesh_cfg'}[sub]  # config.py:160-176
        if cfg.get(sub) and key in cfg:
            cfg.merge(cfg[key])
            cfg.merge_from_list(list(opts))
    if cfg.num_latent_code < 0:
        cfg.num_latent_code = cfg.num_train_frame
    return cfg


class LayeredCfg:
    """Live view of the reference's global ``lib.config.cfg`` (yacs) over this package's defaults:
    a key the reference sets (its yaml, CLI pairs, run.py:50's ``cfg.perturb = 0`` made after the
    plugins were built) wins; a key only this backend defines (``render_precision``, ``chunk`` ...)
    comes from the defaults. Attribute reads and ``get`` are resolved on every access."""

    def __init__(self, ref, base):
        object.__setattr__(self, '_ref', ref)
        object.__setattr__(self, '_base', base)

    def __getattr__(self, name):
        ref = object.__getattribute__(self, '_ref')
        if name in ref:
            return ref[name]
        base = object.__getattribute__(self, '_base')
        if name in base:
            return base[name]
        raise AttributeError(name)

    def __setattr__(self, name, value):
        self._ref[name] = value

    def __contains__(self, name):
        return name in self._ref or name in self._base

    def __getitem__(self, name):
        try:
            return self.__getattr__(name)
        except AttributeError as e:
            raise KeyError(name) from e

    def get(self, name, default=None):
        try:
            return self.__getattr__(name)
        except AttributeError:
            return default


def active():
    """The configuration a plugin built without an explicit cfg reads: the reference's global
    ``lib.config.cfg`` when the reference's config module is loaded (its factories call
    ``Network()``, ``Renderer(net)``, ``NetworkWrapper(net)`` with no cfg: make_network.py:5-9,
    make_renderer.py:5-9, make_trainer.py:5-14), else this package's ``cfg``."""
    import sys
    mod = sys.modules.get('lib.config')
    ref = getattr(mod, 'cfg', None) if mod is not None else None
    if ref is None:
        return cfg
    return LayeredCfg(ref, cfg)


cfg = defaults()
