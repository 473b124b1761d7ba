"""Seeded synthetic weights for ``BlockBasedImgCompLossyNetv9`` and checkpoint loading.

There are no trained checkpoints offline, and torch's default init gives degenerate
latents (every symbol 0, every scale index 0: SURVEY §0.8).  ``synth_state_dict`` draws every
trainable tensor from ``numpy.random.default_rng(seed)`` in the reference's state-dict order
(``Arch.param_shapes``) and scales them so that symbols and scale indexes are non-trivial:

* transform convs: N(0, 1/fan_in_live) -- unit gain through the GDN chain;
* ``prtr_forward3.5`` (last encoder conv) x ``Y_GAIN`` so latents span several quantisation bins;
* ``prtr_inverse1`` x ``YQ_GAIN`` and ``prtr_inverse3.5`` x ``XHAT_GAIN`` so the IGDN chain stays O(1)
  and reconstructions mostly stay inside the clamp;
* ``get_meanscale.6`` scale half: bias = exp(linspace(-2, 5, M)) so the scale index spans the table;
* GDN: beta_eff ~ U(0.5, 1.5), gamma_eff = 0.1 I + U(0, 0.5)/C; stored through the reference's
  ``NonNegativeParametrizer.init`` (utils/parametrizers.py:42-43) so that the forward reparam
  (:45-47) gives back beta_eff / gamma_eff.

``rate="low"`` draws the same tensors and re-scales them to the B8_lowrate operating point (about
0.12-0.14 bpp on uniform-noise frames, BASELINE.md: the published B8_lowrate point is 0.117 bpp): small
latents (``LOW_Y_GAIN``), a context net whose scale channels mostly sit at the bottom of the scale
table with a few wide ones (bias exp(-2.6 + 3.6 (i/(M-1))^18)), weak mean prediction.  Almost every
symbol is 0, as in a trained low-rate model, which is the regime the rANS decoder sees on that config.

The same function feeds the reference (golden generation), the oracle, the HIP library and bench.py,
so all of them see identical weights for a seed.
"""
from __future__ import annotations

import math
from typing import Dict

import numpy as np

from .arch import Arch

PEDESTAL = float(2.0 ** -18) ** 2          # NonNegativeParametrizer reparam_offset**2, utils/parametrizers.py:36
Y_GAIN = 8.0
XHAT_GAIN = 0.6
YQ_GAIN = 0.12
MEAN_GAIN = 0.5
# rate="low" (B8_lowrate operating point)
LOW_Y_GAIN = 0.4
LOW_SCALE_GAIN = 0.3
LOW_MEAN_GAIN = 0.1
LOW_SCALE_POW = 18.0


def synth_state_dict(arch: Arch, seed: int = 1337, rate: str = "high") -> Dict[str, np.ndarray]:
    if rate not in ("high", "low"):
        raise ValueError(f"rate must be 'high' or 'low', not {rate!r}")
    low = rate == "low"
    rng = np.random.default_rng(seed)
    out: Dict[str, np.ndarray] = {}
    convs = {c[0]: c for c in arch.conv_specs()}
    for name, shape in arch.param_shapes():
        mod, leaf = name.rsplit(".", 1)
        if leaf == "weight":
            _, mtype, cin, cout, k = convs[mod]
            live = cin * (4 if (k == 3 and mtype == "A") else 5 if k == 3 else 1)
            w = rng.standard_normal(shape, dtype=np.float32) * np.float32(1.0 / math.sqrt(live))
            if mod == "prtr_forward3.5":
                w *= np.float32(LOW_Y_GAIN if low else Y_GAIN)
            if mod == "prtr_inverse1":
                w *= np.float32(YQ_GAIN)
            if mod == "prtr_inverse3.5":
                w *= np.float32(XHAT_GAIN)
            if mod == "get_meanscale.6":
                w[: arch.M] *= np.float32(LOW_SCALE_GAIN if low else 1.5)   # scale channels around the bias
                w[arch.M:] *= np.float32(LOW_MEAN_GAIN if low else MEAN_GAIN)   # mean channels
            out[name] = w
        elif leaf == "bias":
            b = (rng.standard_normal(shape, dtype=np.float32) * np.float32(0.05))
            if mod == "get_meanscale.6":
                if low:
                    t = np.arange(arch.M, dtype=np.float64) / max(arch.M - 1, 1)
                    b[: arch.M] = np.exp(-2.6 + 3.6 * t ** LOW_SCALE_POW).astype(np.float32)
                else:
                    b[: arch.M] = np.exp(np.linspace(-2.0, 5.0, arch.M)).astype(np.float32)
            out[name] = b
        elif leaf == "beta":
            beta_eff = rng.uniform(0.5, 1.5, size=shape).astype(np.float32)
            out[name] = np.sqrt(np.maximum(beta_eff + np.float32(PEDESTAL), np.float32(PEDESTAL))).astype(np.float32)
        elif leaf == "gamma":
            c = shape[0]
            g = (rng.uniform(0.0, 1.0, size=shape) * (0.5 / c)).astype(np.float32)
            g[np.arange(c), np.arange(c)] += np.float32(0.1)
            out[name] = np.sqrt(np.maximum(g + np.float32(PEDESTAL), np.float32(PEDESTAL))).astype(np.float32)
        else:  # pragma: no cover
            raise KeyError(name)
    return out


def load_reference_checkpoint(path: str) -> Dict[str, np.ndarray]:
    """Load an eval checkpoint in the reference's format ({'state_dict0': sd} or a full training
    checkpoint, agents/base.py:89-128; experiments/extract_model_weights_only.py:20-28) with the safe
    loader only (``weights_only=True``)."""
    import torch
    ck = torch.load(path, map_location="cpu", weights_only=True)
    sd = ck["state_dict0"] if "state_dict0" in ck else ck
    return {k: v.detach().cpu().numpy() for k, v in sd.items()}
