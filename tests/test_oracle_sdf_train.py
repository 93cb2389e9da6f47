"""CPU: pin the sdf_pdf training restatement (oracle/restate_sdf.py render_train + loss_terms) to the
reference's own training step (tests/golden/g13_sdf_train.npz from oracle/gen_goldens.py --sdf-train:
tpose_trainer.NetworkWrapper over anisdf_pdf_network.Network, loss.backward(), the KNN stub as in
G6/G7). Losses, every scalar stat, the observed-gradient rows and the kept parameter gradients
(second-order terms included: the eikonal, observed-gradient and normal-to-colour paths)."""
import numpy as np
import torch

from oracle import restate_sdf

from ._common import assert_golden_equal, golden, oracle_params_sdf

torch.set_num_threads(1)


def g13_batch(g):
    keys = ('ray_o', 'ray_d', 'near', 'far', 'occupancy', 'mask_at_box', 'rgb', 'A', 'big_A', 'R', 'Th', 'poses',
            'pvertices', 'weights', 'tbounds', 'latent_index')
    b = {k: torch.from_numpy(np.ascontiguousarray(g[k])) for k in keys}
    b['iter_step'] = int(g['iter_step'])
    return b


def oracle_step(g):
    P = {k: v.requires_grad_() for k, v in oracle_params_sdf().items()}
    b = g13_batch(g)
    ret = restate_sdf.render_train(P, b, t_rand=torch.from_numpy(g['t_rand']))
    loss, stats = restate_sdf.loss_terms(ret, b)
    loss.backward()
    return P, ret, loss, stats, b


def test_g13_sdf_training_step_matches_reference():
    g = golden('g13_sdf_train')
    P, ret, loss, stats, b = oracle_step(g)
    assert int(ret['resd'].shape[1]) == int(g['n_kept'])
    assert int(ret['observed_gradients'].shape[1]) == int(g['n_observed']) > 0
    assert int(ret['msk_sdf'].shape[1]) == int(g['msk_len'])
    assert_golden_equal(b['tbounds'].numpy(), g['tbounds_after'], err_msg='tbounds widened in place')
    assert_golden_equal(loss.detach().numpy(), g['loss'], err_msg='loss', rtol=1e-4)
    for k in ('offset_loss', 'grad_loss', 'ograd_loss', 'mask_loss', 'img_loss'):
        assert_golden_equal(stats[k].detach().numpy(), g['stat_' + k], err_msg=k, rtol=1e-4)
    assert sorted(k for k, v in P.items() if v.grad is not None) == sorted(g['grad_keys'].tolist())
    n = 0
    for key in g.files:
        if not key.startswith('grad_') or key == 'grad_keys':
            continue
        name = key[5:]
        ref = g[key]
        got = P[name].grad.numpy()
        # second-order sums reassociate across CPU dispatches: 1e-4 of the tensor's largest gradient
        assert_golden_equal(got, ref, err_msg=name, rtol=1e-4, atol=1e-4 * float(np.abs(ref).max()) + 1e-12)
        n += 1
    assert n >= 40
