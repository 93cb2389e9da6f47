"""Checkpoint format compatibility: the reference's
``lib/utils/net_utils.py:288-396`` (``load_model``, ``save_model``, ``load_network``).

A reference ``latest.pth`` / ``{epoch}.pth`` is a dict ``{'net', 'optim', 'scheduler', 'recorder',
'epoch'}``; ``Network`` / ``network_sdf.Network`` keep the reference state_dict names, so the
``net`` entry loads strictly. Files are read with ``torch.load(weights_only=True)`` (tensors,
numbers, strings and containers only — nothing from the file is executed).

``FusedStep`` (trainer.py) keeps Adam's moments in flat blobs; ``adam_state_dict`` /
``load_adam_state_dict`` convert them to and from ``torch.optim.Adam``'s state_dict with one
parameter group per tensor (``lib/train/optimizer.py:12-27``), so a run can move between the
reference trainer and the fused step in either direction.
"""
import os

import torch


def _pick(model_dir, epoch):
    if os.path.isdir(model_dir):
        names = os.listdir(model_dir)
        pths = [int(p.split('.')[0]) for p in names if p != 'latest.pth' and p.endswith('.pth')]
        if not pths and 'latest.pth' not in names:
            return None
        if epoch == -1:
            pth = 'latest' if 'latest.pth' in names else max(pths)
        else:
            pth = epoch
        return os.path.join(model_dir, f'{pth}.pth')
    return model_dir


def load_network(net, model_dir, resume=True, epoch=-1, strict=True, only=()):
    """net_utils.py:357-396: returns the next epoch (0 when nothing was loaded)."""
    if not resume or not os.path.exists(model_dir):
        return 0
    path = _pick(model_dir, epoch)
    if path is None:
        return 0
    ckpt = torch.load(path, map_location='cpu', weights_only=True)
    sd = ckpt['net']
    if only:
        strict = False
        sd = {k: v for k, v in sd.items() if any(k.startswith(o) for o in only)}
    dev = next(net.parameters()).device
    net.load_state_dict({k: v.to(dev) for k, v in sd.items()}, strict=strict)
    net._anr_weights_epoch = getattr(net, '_anr_weights_epoch', 0) + 1  # packed weights are stale
    return ckpt['epoch'] + 1


def load_model(net, optim_state_target, scheduler, recorder, model_dir, resume=True, epoch=-1):
    """net_utils.py:288-323. ``optim_state_target``: a torch optimizer or a FusedStep."""
    if not resume or not os.path.exists(model_dir):
        return 0
    path = _pick(model_dir, epoch)
    if path is None:
        return 0
    ckpt = torch.load(path, map_location='cpu', weights_only=True)
    dev = next(net.parameters()).device
    net.load_state_dict({k: v.to(dev) for k, v in ckpt['net'].items()})
    net._anr_weights_epoch = getattr(net, '_anr_weights_epoch', 0) + 1
    if hasattr(optim_state_target, 'load_adam_state_dict'):
        optim_state_target.load_adam_state_dict(ckpt['optim'])
    else:
        optim_state_target.load_state_dict(ckpt['optim'])
    if scheduler is not None:
        scheduler.load_state_dict(ckpt['scheduler'])
    if recorder is not None:
        recorder.load_state_dict(ckpt['recorder'])
    return ckpt['epoch'] + 1


def save_model(net, optim, scheduler_state, recorder_state, model_dir, epoch, last=False):
    """net_utils.py:326-348 (keeps at most 20 numbered files)."""
    os.makedirs(model_dir, exist_ok=True)
    optim_sd = optim.adam_state_dict() if hasattr(optim, 'adam_state_dict') else optim.state_dict()
    model = {'net': net.state_dict(), 'optim': optim_sd, 'scheduler': scheduler_state, 'recorder': recorder_state,
             'epoch': epoch}
    torch.save(model, os.path.join(model_dir, 'latest.pth' if last else f'{epoch}.pth'))
    pths = sorted(int(p.split('.')[0]) for p in os.listdir(model_dir) if p != 'latest.pth' and p.endswith('.pth'))
    if len(pths) > 20:
        os.remove(os.path.join(model_dir, f'{pths[0]}.pth'))


def adam_state_dict(params, m, v, step, lr, betas, eps, weight_decay):
    """Flat Adam moments -> torch.optim.Adam state_dict with one group per tensor."""
    state, groups, off = {}, [], 0
    for i, p in enumerate(params):
        k = p.numel()
        if step > 0:
            state[i] = {'step': torch.tensor(float(step)), 'exp_avg': m[off:off + k].view_as(p).detach().cpu().clone(),
                        'exp_avg_sq': v[off:off + k].view_as(p).detach().cpu().clone()}
        groups.append({'lr': lr, 'betas': betas, 'eps': eps, 'weight_decay': weight_decay, 'amsgrad': False,
                       'maximize': False, 'foreach': None, 'capturable': False, 'differentiable': False,
                       'fused': None, 'initial_lr': lr, 'params': [i]})
        off += k
    return {'state': state, 'param_groups': groups}


def load_adam_state_dict(sd, params, m, v):
    """torch.optim.Adam state_dict -> flat moments (in place); returns (step, lr of group 0)."""
    off, step = 0, 0
    for i, p in enumerate(params):
        k = p.numel()
        st = sd['state'].get(i, sd['state'].get(str(i)))
        if st is not None:
            m[off:off + k].copy_(st['exp_avg'].reshape(-1))
            v[off:off + k].copy_(st['exp_avg_sq'].reshape(-1))
            step = int(float(st['step']))
        else:
            m[off:off + k].zero_()
            v[off:off + k].zero_()
        off += k
    return step, sd['param_groups'][0]['lr']
