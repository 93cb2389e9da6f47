"""CPU: ResidentFrames (per-image H2D of the blend-weight volumes): a frame's
per-frame tensors are transferred once and reused by later batches of that frame; per-ray keys and
the in-place-widened tbounds travel with every batch."""
import numpy as np
import pytest
import torch

from animatable_nerf_amd.data import ResidentFrames

from ._common import scene


def _batch(frame, seed):
    sc = scene(0.05)
    ro, rd = sc.box_rays(16, seed=seed)
    b = sc.batch_arrays(ro, rd, np.ones(16, np.float32), np.full(16, 2.0, np.float32))
    b['frame_index'] = np.array([frame])
    b['pbw'] = b['pbw'] + np.float32(frame)  # a different volume per frame
    return b


def test_frames_upload_once_and_are_reused():
    rf = ResidentFrames('cpu')
    b0 = _batch(3, 1)
    d0 = rf.to_device(b0)
    n_keys = sum(1 for k in ResidentFrames.KEYS if k in b0)
    assert rf.uploads == n_keys
    d1 = rf.to_device(_batch(3, 2))                      # same frame, other rays
    assert rf.uploads == n_keys
    for k in ResidentFrames.KEYS:
        assert d1[k] is d0[k]
        assert np.array_equal(d0[k].numpy(), b0[k])
    assert not torch.equal(d0['ray_d'], d1['ray_d'])     # per-ray keys are fresh
    assert d1['tbounds'] is not d0['tbounds']            # not cached (widened in place by sdf_pdf)
    d2 = rf.to_device(_batch(4, 1))                      # another frame
    n_frame = sum(1 for k in ResidentFrames.KEYS if k in b0 and k not in ResidentFrames.SUBJECT_KEYS)
    assert rf.uploads == n_keys + n_frame                # subject keys (tbw) are not uploaded again
    assert not torch.equal(d2['pbw'], d0['pbw'])
    assert d2['tbw'] is d0['tbw']
    per_frame = sum(d0[k].numel() * d0[k].element_size() for k in ResidentFrames.KEYS if k in b0)
    subject = sum(d0[k].numel() * d0[k].element_size() for k in ResidentFrames.SUBJECT_KEYS if k in b0)
    assert rf.resident_bytes() == 2 * per_frame - subject


def test_mixed_frame_batch_is_refused():
    rf = ResidentFrames('cpu')
    b = _batch(3, 1)
    b['frame_index'] = np.array([3, 5])
    with pytest.raises(ValueError, match='one frame'):
        rf.to_device(b)
    b['frame_index'] = np.array([3, 3])                  # several images of one frame are fine
    rf.to_device(b)
