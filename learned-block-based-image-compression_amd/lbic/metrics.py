"""Image-quality metrics of eval_model (agents/blkbsdimgcomp_agent.py:608-619).

MS-SSIM: the reference calls ``pytorch_msssim.ms_ssim(x, y, data_range=1.0)`` (absent here).  This is the
standard definition that package implements (Wang et al. 2003): 11-tap Gaussian window, sigma 1.5,
K1 = 0.01, K2 = 0.03, 5 scales with weights (0.0448, 0.2856, 0.3001, 0.2363, 0.1333), 2x2 average
pooling between scales, mean over channels; "parity unpinned" (no fixture of the package's output).
"""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F

MS_WEIGHTS = (0.0448, 0.2856, 0.3001, 0.2363, 0.1333)


def _gauss(size=11, sigma=1.5, device=None):
    c = torch.arange(size, dtype=torch.float32, device=device) - size // 2
    g = torch.exp(-(c ** 2) / (2 * sigma ** 2))
    return g / g.sum()


def _filt(x, g):
    C = x.shape[1]
    x = F.conv2d(x, g.view(1, 1, 1, -1).repeat(C, 1, 1, 1), groups=C)
    return F.conv2d(x, g.view(1, 1, -1, 1).repeat(C, 1, 1, 1), groups=C)


def _ssim(x, y, g, data_range):
    C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    mu1, mu2 = _filt(x, g), _filt(y, g)
    s11 = _filt(x * x, g) - mu1 ** 2
    s22 = _filt(y * y, g) - mu2 ** 2
    s12 = _filt(x * y, g) - mu1 * mu2
    cs = (2 * s12 + C2) / (s11 + s22 + C2)
    ssim = ((2 * mu1 * mu2 + C1) / (mu1 ** 2 + mu2 ** 2 + C1)) * cs
    return ssim.flatten(2).mean(-1), cs.flatten(2).mean(-1)


def ms_ssim(x, y, data_range=1.0):
    """NaN for frames smaller than 161 px a side (pytorch_msssim refuses those: 5 scales x 11-tap window)."""
    if min(x.shape[-2:]) <= (11 - 1) * 2 ** 4:
        return torch.tensor(float("nan"))
    g = _gauss(device=x.device)
    w = torch.tensor(MS_WEIGHTS, device=x.device)
    mcs = []
    for i in range(len(MS_WEIGHTS)):
        ssim, cs = _ssim(x, y, g, data_range)
        if i < len(MS_WEIGHTS) - 1:
            mcs.append(torch.relu(cs))
            pad = [s % 2 for s in x.shape[2:]]
            x = F.avg_pool2d(x, 2, padding=pad)
            y = F.avg_pool2d(y, 2, padding=pad)
    ssim = torch.relu(ssim)
    vals = torch.stack(mcs + [ssim], dim=0)
    return torch.prod(vals ** w.view(-1, 1, 1), dim=0).mean()


def psnr_from_mse(mse):
    return -10 * math.log10(mse)
