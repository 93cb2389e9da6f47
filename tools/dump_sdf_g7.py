"""Debug helper: render the G7 rays on the GPU and save the outputs (gpurun_out/sdf_g7.npz)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from tests._common import make_net_sdf, pdf_batch_np, pdf_g7_rays, pdf_scene, sdf_cfg, to_torch  # noqa: E402
from animatable_nerf_amd.renderer_sdf import Renderer  # noqa: E402

dev = torch.device('cuda:0')
net = make_net_sdf(dev)
net.train()
r = Renderer(net, sdf_cfg())
ro, rd = pdf_g7_rays()
b, _ = pdf_batch_np(pdf_scene(), ro, rd)
ret = r.render_device(to_torch(b, dev))
os.makedirs('gpurun_out', exist_ok=True)
np.savez_compressed('gpurun_out/sdf_g7.npz', **{k: v.cpu().numpy() for k, v in ret.items()})
print('saved', {k: tuple(v.shape) for k, v in ret.items()})
