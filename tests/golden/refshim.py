"""Import the reference's own model code from /root/reference (THIS container only; golden generation).

Test infrastructure, not product code: only ``gen_golden.py`` uses it, and nothing on the GPU box does
(the reference does not travel).  Mechanism:

* ``utils``, ``graphs``, ``graphs.layers``, ``graphs.models`` are registered as namespace modules
  pointing at the reference directories, so their auto-import ``__init__`` files (which pull in
  torchvision / easydict / pytorch_msssim, absent here) never run;
* ``compressai`` (not installed, not vendored) is mapped onto the reference's own in-tree copies:
  ``compressai.layers.GDN`` -> graphs/layers/gdn_compressai.py:26,
  ``compressai.entropy_models.GaussianConditional`` -> graphs/layers/entropy_layers_cai.py:517,
  ``compressai.ops.LowerBound`` -> utils/bound_ops.py:45;
* the two C++ pieces of CompressAI are NOT stood in for: ``_CXX.pmf_to_quantized_cdf`` records the
  float pmf the reference hands it (graphs/layers/entropy_layers_cai.py:61-64) and returns a
  placeholder, and ``ans.BufferedRansEncoder`` records the (symbol, index) lists the reference hands
  it (graphs/models/BlockBasedImgCompLossy_net.py:353-360) and returns an empty string.  So the golden
  vectors pin everything up to the coder's inputs; CDF tables and bitstream bytes stay "parity
  unpinned" (SURVEY §8c.4).  ``ans.RansDecoder`` replays recorded symbols, which runs the
  reference's decompress() loop teacher-forced.
"""
from __future__ import annotations

import sys
import types

REF = "/root/reference"

PMF_LOG = []          # float pmfs handed to pmf_to_quantized_cdf
ENC_LOG = []          # (symbols, indexes) handed to BufferedRansEncoder.encode_with_indexes
DEC_QUEUE = []        # symbol chunks RansDecoder.decode_stream returns (in order)
DEC_IDX_LOG = []      # indexes the reference decoder asked for


def _ns(name, path):
    m = types.ModuleType(name)
    m.__path__ = [path]
    sys.modules[name] = m
    return m


class _RecEncoder:
    def __init__(self):
        self.syms, self.idxs = [], []

    def encode_with_indexes(self, symbols, indexes, cdf, cdf_lengths, offsets):
        self.syms.extend(symbols)
        self.idxs.extend(indexes)
        ENC_LOG.append((list(symbols), list(indexes)))

    def flush(self):
        return b""


class _ReplayDecoder:
    def set_stream(self, s):
        pass

    def decode_stream(self, indexes, cdf, cdf_lengths, offsets):
        DEC_IDX_LOG.append(list(indexes))
        return DEC_QUEUE.pop(0)


def install():
    if "graphs.models.BlockBasedImgCompLossy_net" in sys.modules:
        return sys.modules["graphs.models.BlockBasedImgCompLossy_net"]
    if REF not in sys.path:
        sys.path.insert(0, REF)
    _ns("utils", REF + "/utils")
    _ns("graphs", REF + "/graphs")
    _ns("graphs.layers", REF + "/graphs/layers")
    _ns("graphs.models", REF + "/graphs/models")

    cai = types.ModuleType("compressai")
    cai.__path__ = []
    sys.modules["compressai"] = cai
    cxx = types.ModuleType("compressai._CXX")

    def pmf_to_quantized_cdf(pmf, precision):
        PMF_LOG.append(list(pmf))
        return [0] * (len(pmf) + 1)

    cxx.pmf_to_quantized_cdf = pmf_to_quantized_cdf
    sys.modules["compressai._CXX"] = cxx
    ans = types.ModuleType("compressai.ans")
    ans.BufferedRansEncoder = _RecEncoder
    ans.RansEncoder = _RecEncoder
    ans.RansDecoder = _ReplayDecoder
    sys.modules["compressai.ans"] = ans
    cai.ans = ans
    cai.available_entropy_coders = lambda: ["ans"]
    cai.get_entropy_coder = lambda: "ans"

    import utils.bound_ops as bound_ops
    ops = types.ModuleType("compressai.ops")
    ops.LowerBound = bound_ops.LowerBound
    sys.modules["compressai.ops"] = ops
    import graphs.layers.entropy_layers_cai as ent
    em = types.ModuleType("compressai.entropy_models")
    em.GaussianConditional = ent.GaussianConditional
    em.EntropyBottleneck = ent.EntropyBottleneck
    sys.modules["compressai.entropy_models"] = em
    import graphs.layers.gdn_compressai as gdn
    lay = types.ModuleType("compressai.layers")
    lay.GDN = gdn.GDN
    lay.GDN1 = gdn.GDN1
    sys.modules["compressai.layers"] = lay
    import graphs.models.BlockBasedImgCompLossy_net as net
    return net


def make_model(arch, sd_numpy):
    """Instantiate the reference v9 net for ``arch`` and load our synthetic parameters into it."""
    import torch
    net = install()
    cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M)
    model = net.BlockBasedImgCompLossyNetv9(cfg)
    missing, unexpected = model.load_state_dict({k: torch.from_numpy(v) for k, v in sd_numpy.items()}, strict=False)
    assert not unexpected, unexpected
    assert all(k.endswith(("mask", "pedestal", "bound", "_offset", "_quantized_cdf", "_cdf_length",
                           "scale_table", "scale_bound")) for k in missing), missing
    model.eval()
    return model, net
