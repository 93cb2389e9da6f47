"""CPU: the animation stage's oracle (lib/train/trainers/
aninerf_animation_trainer.py): oracle/restate.anim_losses with autograd vs the reference run
(golden G11: 4096 points per path, rotated world frame) — losses and novel_pose_bw gradients
bit-exact at one thread on a host with the generating host's CPU kernels, else within fp32
roundoff (tests/_common.assert_golden_equal)."""
import numpy as np
import torch

from ._common import assert_golden_equal, golden, state_dict_novel_np

G11_GRADS = ('bw_latent.weight', 'bw_linears.0.weight', 'bw_linears.0.bias', 'bw_linears.4.bias',
             'bw_linears.5.bias', 'bw_linears.7.weight', 'bw_linears.7.bias', 'bw_fc.weight', 'bw_fc.bias')


def g11_inputs():
    g = golden('g11_anim')
    keys = ('A', 'pbw', 'tbw', 'pbounds', 'wbounds', 'tbounds', 'R', 'Th', 'bw_latent_index', 'latent_index')
    batch = {k: torch.from_numpy(np.ascontiguousarray(g[k])) for k in keys}

    def pts(bounds, vals):  # get_sampling_points (aninerf_animation_trainer.py:143-160)
        lo, hi = bounds[:, 0], bounds[:, 1]
        return (hi - lo)[:, None] * torch.from_numpy(vals) + lo[:, None]

    return g, batch, pts(batch['wbounds'], g['wvals']), pts(batch['tbounds'], g['tvals'])


def test_anim_oracle_matches_reference():
    from oracle import restate
    torch.set_num_threads(1)
    g, batch, wpts, tpts = g11_inputs()
    P = {k: torch.from_numpy(v.copy()).requires_grad_(k.startswith('novel_pose_bw.'))
         for k, v in state_dict_novel_np().items()}
    loss, l0, l1 = restate.anim_losses(P, batch, wpts, tpts, norm_th=float(g['norm_th']),
                                       train_th=float(g['train_th']))
    loss.backward()
    assert_golden_equal(np.float32(loss.item()), g['loss'], 'loss')
    assert_golden_equal(np.float32(l0.item()), g['bw_loss0'], 'bw_loss0')
    assert_golden_equal(np.float32(l1.item()), g['bw_loss1'], 'bw_loss1')
    for k in G11_GRADS:
        gr = P['novel_pose_bw.' + k].grad.numpy()
        if k == 'bw_latent.weight':
            gr = gr[int(g['bw_latent_index'][0])]
        assert_golden_equal(gr, g['grad_' + k], k)
