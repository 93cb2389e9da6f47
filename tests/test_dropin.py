"""CPU: the plugins load the way the reference's factories load them and read the reference's
configuration.

* ``make_network`` / ``make_renderer`` / ``make_trainer`` call ``imp.load_source(module, path)`` and
  then ``Network()``, ``Renderer(net)``, ``NetworkWrapper(net)`` with no cfg (make_network.py:5-9,
  make_renderer.py:5-9, make_trainer.py:5-14). A stand-in ``lib.config`` module holding the
  reference's global ``cfg`` is put in ``sys.modules`` (as ``import lib.config`` does in train_net.py /
  run.py), and the plugins must size themselves from it (aninerf_313: num_train_frame 60) and see its
  later edits (run.py:50 sets ``cfg.perturb = 0`` after the network is built).
* The state_dict names and shapes match the reference Network of every config BASELINE.json names
  (golden G13, dumped by oracle/gen_goldens.py --state-dicts from the real reference), so
  ``load_network(strict=True)`` reads its checkpoints.
No compute calls (no GPU)."""
import imp
import json
import os
import sys
import types

import pytest

from animatable_nerf_amd import config

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, 'animatable_nerf_amd')
G13 = os.path.join(ROOT, 'tests', 'golden', 'g13_state_dicts.json')


def _reference_cfg(**kw):
    """a yacs-like CfgNode with the keys the reference's config.py / yaml give (no backend-only keys)"""
    c = config.CfgNode({'N_samples': 64, 'N_rand': 1024, 'perturb': 1, 'norm_th': 0.05, 'train_th': 0.0,
                        'num_train_frame': 260, 'num_eval_frame': 133, 'num_latent_code': 260,
                        'aninerf_animation': False, 'test_novel_pose': False, 'white_bkgd': False,
                        'tpose_viewdir': True,
                        'train': {'lr': 5e-4, 'weight_decay': 0.0, 'optim': 'adam'}})
    c.update(kw)
    return c


@pytest.fixture
def ref_cfg(monkeypatch):
    cfg = _reference_cfg(num_train_frame=60, num_latent_code=60, num_eval_frame=1000)  # configs/aninerf_313.yaml
    lib = types.ModuleType('lib')
    lib.__path__ = []
    libcfg = types.ModuleType('lib.config')
    libcfg.cfg = cfg
    lib.config = libcfg
    monkeypatch.setitem(sys.modules, 'lib', lib)
    monkeypatch.setitem(sys.modules, 'lib.config', libcfg)
    # imp.load_source replaces the package's modules: restore them after the test
    for m in ('network', 'renderer', 'trainer', 'network_sdf', 'renderer_sdf'):
        name = 'animatable_nerf_amd.' + m
        __import__(name)
        monkeypatch.setitem(sys.modules, name, sys.modules[name])
    return cfg


def _load(module):
    # the reference's factories: imp.load_source(cfg.network_module, cfg.network_path)
    return imp.load_source('animatable_nerf_amd.' + module, os.path.join(PKG, module + '.py'))


def test_plugins_read_the_reference_cfg(ref_cfg):
    net = _load('network').Network()
    assert tuple(net.tpose_human.nf_latent.weight.shape) == (60, 128)
    assert tuple(net.bw_latent.weight.shape) == (61, 128)
    renderer = _load('renderer').Renderer(net)
    assert renderer.cfg.N_samples == 64 and renderer.cfg.perturb == 1
    assert renderer.cfg.get('render_precision') == 'fp32'  # a backend-only key: the package default
    ref_cfg.perturb = 0  # run.py:50, after make_network
    assert renderer.cfg.perturb == 0
    wrapper = _load('trainer').NetworkWrapper(net)
    assert wrapper.renderer.cfg.perturb == 0 and wrapper.renderer.cfg.num_train_frame == 60
    # the eval renderer draws no stratification noise at perturb 0 even in train() mode (run.py:58)
    import torch
    net.train()
    assert renderer._t_rand(8, torch.device('cpu'), None) is None
    ref_cfg.perturb = 1
    assert renderer._t_rand(8, torch.device('cpu'), None).shape == (8, 64)


def test_sdf_plugins_read_the_reference_cfg(ref_cfg):
    net = _load('network_sdf').Network()
    sd = net.state_dict()
    assert tuple(sd['resd_latent.weight'].shape) == (60, 128)
    assert tuple(sd['tpose_human.color_network.color_latent.weight'].shape) == (60, 128)
    r = _load('renderer_sdf').Renderer(net)
    ref_cfg.perturb = 0
    assert r.cfg.perturb == 0


def test_no_reference_loaded_means_package_cfg():
    assert 'lib.config' not in sys.modules or not hasattr(sys.modules['lib.config'], 'cfg')
    assert config.active() is config.cfg


@pytest.mark.parametrize('name', ['s9p', '313', 's9p_animation', 'sdf_pdf_s9p'])
def test_state_dict_matches_reference(name):
    g = json.load(open(G13))[name]
    cfg = config.defaults()
    cfg.num_train_frame = g['num_train_frame']
    cfg.num_eval_frame = g['num_eval_frame']
    cfg.num_latent_code = g['num_latent_code']
    if 'aninerf_animation' in g['opts']:
        cfg.aninerf_animation = True
    if name.startswith('sdf'):
        from animatable_nerf_amd import network_sdf
        net = network_sdf.Network(cfg)
    else:
        from animatable_nerf_amd import network
        net = network.Network(cfg)
    ours = [[k, list(v.shape)] for k, v in net.state_dict().items()]
    assert ours == g['state_dict']


@pytest.mark.parametrize('name,subject', [('s9p', 'aninerf_s9p'), ('313', 'aninerf_313'),
                                          ('sdf_pdf_s9p', 'anisdf_pdf_s9p')])
def test_subject_presets_match_reference_cfg(name, subject):
    """config.subject(...) (used by the GPU tests and bench.py, where the yaml files are absent) sizes the
    networks as the reference's own cfg of that experiment does (golden G13: its yaml run through lib.config)."""
    g = json.load(open(G13))[name]
    cfg = config.subject(subject)
    for k in ('num_train_frame', 'num_eval_frame', 'num_latent_code'):
        assert cfg[k] == g[k], (k, cfg[k], g[k])
    if name.startswith('sdf'):
        from animatable_nerf_amd import network_sdf
        net = network_sdf.Network(cfg)
    else:
        from animatable_nerf_amd import network
        net = network.Network(cfg)
    assert [[k, list(v.shape)] for k, v in net.state_dict().items()] == g['state_dict']
