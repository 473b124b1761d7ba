"""Block <-> channel layout (agents/blkbsdimgcomp_agent.py:853-873).

The reference arranges an image [1, 3, H, W] as [1, 3B^2, H/B, W/B] with channel index
(py*B + px)*3 + colour.  The HIP path stores the same channels block-major, [n, H/B, W/B, 3B^2], so one
block's channel vector is contiguous (coalesced loads).  Pure data movement, no arithmetic.
"""
from __future__ import annotations

import numpy as np
import torch


def image_to_blocks(img_chw: np.ndarray, B: int) -> np.ndarray:
    """[3, H, W] -> block-major [H/B, W/B, 3B^2]."""
    C, H, W = img_chw.shape
    x = img_chw.reshape(C, H // B, B, W // B, B)                 # c, vb, py, hb, px
    return np.ascontiguousarray(x.transpose(1, 3, 2, 4, 0).reshape(H // B, W // B, B * B * C))


def blocks_to_image(xb: np.ndarray, B: int) -> np.ndarray:
    Hb, Wb, CC = xb.shape
    C = CC // (B * B)
    return np.ascontiguousarray(xb.reshape(Hb, Wb, B, B, C).transpose(4, 0, 2, 1, 3).reshape(C, Hb * B, Wb * B))


def arrange_block_pixels_to_channel_dim(x: torch.Tensor, B: int, dev=None) -> torch.Tensor:
    """[n, 3, H, W] -> [n, 3B^2, H/B, W/B] (agents/blkbsdimgcomp_agent.py:853-860)."""
    n, C, H, W = x.shape
    y = x.reshape(n, C, H // B, B, W // B, B).permute(0, 3, 5, 1, 2, 4)   # n, py, px, c, vb, hb
    return y.reshape(n, B * B * C, H // B, W // B).contiguous()


def arrange_channel_dim_to_block_pixels(y: torch.Tensor, B: int, dev=None) -> torch.Tensor:
    """[n, 3B^2, H/B, W/B] -> [n, 3, H, W] (agents/blkbsdimgcomp_agent.py:863-873)."""
    n, CC, Hb, Wb = y.shape
    C = CC // (B * B)
    x = y.reshape(n, B, B, C, Hb, Wb).permute(0, 3, 4, 1, 5, 2)           # n, c, vb, py, hb, px
    return x.reshape(n, C, Hb * B, Wb * B).contiguous()
