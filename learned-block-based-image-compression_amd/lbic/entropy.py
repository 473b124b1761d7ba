"""Host-side mirror of the reference's conditional Gaussian entropy model (``GaussianConditional``,
graphs/layers/entropy_layers_cai.py:517-654, the class the model uses through
``compressai.entropy_models``).

Only the once-per-model table build lives here (``update``): the scale table and pmfs are computed with
the same torch CPU ops as the reference (bit-identical), and the 16-bit quantized CDFs by the native
``lbc_pmf_to_quantized_cdf`` (replacing CompressAI's C++ ``pmf_to_quantized_cdf``).  Per-latent
quantisation, scale indexing and likelihood run inside the HIP kernels (kernels.hip, EPI_QUANT).
"""
from __future__ import annotations

import math

import numpy as np
import torch

from . import _lib

SCALES_MIN, SCALES_MAX, SCALES_LEVELS = 0.11, 256, 64   # net:13-18


def get_scale_table(mmin=SCALES_MIN, mmax=SCALES_MAX, levels=SCALES_LEVELS):
    """net:13-18."""
    return torch.exp(torch.linspace(math.log(mmin), math.log(mmax), levels))


def pmf_to_quantized_cdf(pmf, precision=16):
    """compressai._CXX.pmf_to_quantized_cdf (entropy_layers_cai.py:61-64) via liblbic.so."""
    p = np.ascontiguousarray(np.asarray(pmf, np.float32))
    out = np.zeros(len(p) + 1, np.uint32)
    _lib.check(_lib.lib().lbc_pmf_to_quantized_cdf(_lib.ptr(p), len(p), precision, _lib.ptr(out)))
    return torch.from_numpy(out.astype(np.int32))


class GaussianConditional:
    """Buffers and ``update`` of the reference's GaussianConditional(None) (scale_bound 0.11,
    tail_mass 1e-9, likelihood bound 1e-9, 16-bit precision)."""

    def __init__(self, scale_bound=0.11, tail_mass=1e-9, precision=16):
        self.scale_bound = float(scale_bound)
        self.tail_mass = float(tail_mass)
        self.entropy_coder_precision = int(precision)
        self.scale_table = torch.Tensor()
        self._offset = torch.IntTensor()
        self._quantized_cdf = torch.IntTensor()
        self._cdf_length = torch.IntTensor()

    @property
    def offset(self):
        return self._offset

    @property
    def quantized_cdf(self):
        return self._quantized_cdf

    @property
    def cdf_length(self):
        return self._cdf_length

    @staticmethod
    def _standardized_cumulative(inputs):
        return 0.5 * torch.erfc(float(-(2 ** -0.5)) * inputs)

    def update_scale_table(self, scale_table, force=False):
        """entropy_layers_cai.py:579-588."""
        if self._offset.numel() > 0 and not force:
            return False
        self.scale_table = torch.Tensor(tuple(float(s) for s in scale_table))
        self.update()
        return True

    def update(self):
        """entropy_layers_cai.py:590-613."""
        from scipy.stats import norm
        multiplier = -norm.ppf(self.tail_mass / 2)
        pmf_center = torch.ceil(self.scale_table * multiplier).int()
        pmf_length = 2 * pmf_center + 1
        max_length = int(torch.max(pmf_length).item())
        samples = torch.abs(torch.arange(max_length).int() - pmf_center[:, None]).float()
        samples_scale = self.scale_table.unsqueeze(1).float()
        upper = self._standardized_cumulative((0.5 - samples) / samples_scale)
        lower = self._standardized_cumulative((-0.5 - samples) / samples_scale)
        pmf = upper - lower
        tail_mass = 2 * lower[:, :1]
        cdf = torch.zeros((len(pmf_length), max_length + 2), dtype=torch.int32)
        for i, p in enumerate(pmf):
            prob = torch.cat((p[: pmf_length[i]], tail_mass[i]), dim=0)
            c = pmf_to_quantized_cdf(prob.numpy(), self.entropy_coder_precision)
            cdf[i, : c.size(0)] = c
        self._quantized_cdf = cdf
        self._offset = -pmf_center
        self._cdf_length = pmf_length + 2

    def _check_cdf_size(self):
        if self._quantized_cdf.numel() == 0:
            raise ValueError("Uninitialized CDFs. Run update() first")
        if len(self._quantized_cdf.size()) != 2:
            raise ValueError(f"Invalid CDF size {self._quantized_cdf.size()}")

    def _check_offsets_size(self):
        if self._offset.numel() == 0:
            raise ValueError("Uninitialized offsets. Run update() first")

    def _check_cdf_length(self):
        if self._cdf_length.numel() == 0:
            raise ValueError("Uninitialized CDF lengths. Run update() first")

    def state_dict(self, prefix="conditional_gaussian_model."):
        return {prefix + "_offset": self._offset, prefix + "_quantized_cdf": self._quantized_cdf,
                prefix + "_cdf_length": self._cdf_length, prefix + "scale_table": self.scale_table,
                prefix + "scale_bound": torch.Tensor([self.scale_bound])}
