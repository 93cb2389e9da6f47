"""Novel-view / pose-sequence renderer over the sdf_pdf network (``lib/networks/renderer/
tpose_renderer_mmsk.py`` as configured by ``configs/sdf_pdf/anisdf_pdf_s9p.yaml:108-139``): the sdf render
with the training-view visibility filter. A sample reaches the network only if it projects inside every
training view's mask (``prepare_inside_pts`` :14-57; batch keys ``Ks``, ``RT``, ``msks``, ``H``, ``W``); the
per-chunk Network.forward call the reference makes on the visible samples (:80-91) is the device render's
chunk: its KNN keep and forced argmin range over them, and ``tbounds`` widens (in place, once) only for
chunks with a visible sample. The filter runs inside the sdf front-end kernel (``anr_sdf_frame.n_views``).
Returns ``rgb_map``, ``acc_map``, ``depth_map`` on the CPU like :124-128.
"""
import torch

from . import renderer_sdf as _renderer_sdf


class Renderer(_renderer_sdf.Renderer):
    visibility_filter = True

    def render(self, batch):
        with torch.no_grad():
            ret = self.render_device(batch)
        return {k: ret[k].cpu() for k in ('rgb_map', 'acc_map', 'depth_map')}
