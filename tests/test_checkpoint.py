"""CPU: checkpoint compatibility with the reference format (net_utils.py:288-396) and the Adam state
conversion between torch.optim.Adam (reference trainer) and FusedStep's flat moments."""
import os

import torch

from animatable_nerf_amd import checkpoint, config, network, trainer

from ._common import make_net


def test_load_network_reference_format(tmp_path):
    src = make_net()
    torch.save({'net': src.state_dict(), 'optim': {}, 'scheduler': {}, 'recorder': {}, 'epoch': 7},
               os.path.join(tmp_path, 'latest.pth'))
    torch.save({'net': src.state_dict(), 'optim': {}, 'scheduler': {}, 'recorder': {}, 'epoch': 3},
               os.path.join(tmp_path, '3.pth'))
    dst = network.Network()
    assert checkpoint.load_network(dst, str(tmp_path)) == 8
    for (k, a), (_, b) in zip(src.state_dict().items(), dst.state_dict().items()):
        assert torch.equal(a, b), k
    assert checkpoint.load_network(network.Network(), str(tmp_path), epoch=3) == 4
    part = network.Network()
    checkpoint.load_network(part, str(tmp_path), only=['bw_linears'])
    assert torch.equal(part.bw_linears[0].weight, src.bw_linears[0].weight)


def test_adam_state_round_trip(tmp_path):
    cfg = config.defaults()
    net = make_net()
    opt = trainer.make_optimizer(cfg, net)
    for p in net.parameters():
        p.grad = torch.randn_like(p) * 1e-2
    opt.step()
    opt.step()
    fs = trainer.FusedStep(make_net(), cfg)
    fs.load_adam_state_dict(opt.state_dict())
    assert fs.t == 2
    sd = fs.adam_state_dict()
    ref = opt.state_dict()
    for i in ref['state']:
        assert torch.equal(sd['state'][i]['exp_avg'], ref['state'][i]['exp_avg'])
        assert torch.equal(sd['state'][i]['exp_avg_sq'], ref['state'][i]['exp_avg_sq'])
    opt2 = trainer.make_optimizer(cfg, make_net())
    opt2.load_state_dict(sd)  # the reference trainer can resume from a FusedStep checkpoint
    checkpoint.save_model(fs.net, fs, {'last_epoch': 1}, {}, str(tmp_path), 1, last=True)
    ck = torch.load(os.path.join(tmp_path, 'latest.pth'), weights_only=True)
    assert set(ck) == {'net', 'optim', 'scheduler', 'recorder', 'epoch'} and ck['epoch'] == 1
