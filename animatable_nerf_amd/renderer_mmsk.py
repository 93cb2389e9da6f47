"""Novel-view / pose-sequence renderer plugin (``lib/networks/renderer/tpose_renderer_mmsk.py``,
SURVEY.md §8(f) row 2): the same device render with the training-view visibility filter —
a sample reaches the network only if it projects inside every training view's mask
(``prepare_inside_pts`` :14-57, batch keys ``Ks``, ``RT``, ``msks``, ``H``, ``W`` of
``tpose_novel_view_dataset.py:191``). The filter runs inside the front-end kernel, before the
prefilter and its per-chunk argmin, which then range over the visible samples as in the reference
(a chunk with no visible sample keeps nothing). Returns ``rgb_map``, ``acc_map``, ``depth_map``
on the CPU like ``:124-128``.
"""
import torch

from . import renderer as _renderer


class Renderer(_renderer.Renderer):
    visibility_filter = True

    def render(self, batch):
        with torch.no_grad():
            ret = self.render_device(batch, bw_rows=False)
        return {k: ret[k].cpu() for k in ('rgb_map', 'acc_map', 'depth_map')}
