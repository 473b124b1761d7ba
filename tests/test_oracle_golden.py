"""Pin the oracle (oracle/oracle.py + oracle/rans_oracle.c) against the reference's own golden vectors.

Tolerances: float activations 1e-5 relative (north_star), symbols / scale indexes bit-exact on the
tie-screened fixtures (tests/golden/gen_golden.py), scale table and pmfs bit-exact / 1 ulp.
"""
import numpy as np
import pytest

from conftest import golden_arch, load_golden, golden_rate
from lbic.weights import synth_state_dict
from oracle import oracle as O

RTOL = 1e-5


def _close(a, b, rtol=RTOL):
    a, b = np.asarray(a, np.float64), np.asarray(b, np.float64)
    scale = max(np.abs(b).max(), 1e-30)
    return np.abs(a - b).max() / scale


def test_scale_table_bit_exact():
    g = load_golden("cdf_pmf")
    assert np.array_equal(O.scale_table().view(np.uint32), g["scale_table"].view(np.uint32))


def test_pmfs_match_reference():
    g = load_golden("cdf_pmf")
    probs, offset, length = O.gaussian_pmfs(g["scale_table"])
    assert np.array_equal(offset, g["offset"])
    assert np.array_equal(length, g["cdf_length"])
    ref = np.split(g["prob"], np.cumsum(g["prob_len"])[:-1])
    for p, r in zip(probs, ref):
        assert p.shape == r.shape
        # scipy erfc (double, rounded) vs torch's float32 erfc: |dp| <= 1e-7 absolute (x 2^16 << 1/2) ...
        assert np.abs(p.astype(np.float64) - r).max() < 1e-7
        # ... and the 16-bit quantized CDFs built from either are identical
        assert np.array_equal(O.pmf_to_quantized_cdf(p), O.pmf_to_quantized_cdf(r))


def test_quantized_cdf_properties():
    """pmf_to_quantized_cdf (CompressAI ops.cpp restated; parity unpinned): monotone, 0..2^16."""
    g = load_golden("cdf_pmf")
    tabs = O.GaussianTables(np.split(g["prob"], np.cumsum(g["prob_len"])[:-1]))
    for i, n in enumerate(tabs.cdf_length):
        c = tabs.cdf[i, :n]
        assert c[0] == 0 and c[-1] == 65536
        assert np.all(np.diff(c) > 0)


def test_rans_roundtrip_with_bypass():
    tabs = O.GaussianTables()
    rng = np.random.default_rng(0)
    idx = rng.integers(0, 64, 5000).astype(np.int32)
    sym = np.rint(rng.standard_normal(5000) * tabs.table[idx] * 1.5).astype(np.int32)
    sym[::97] = 10000                      # far outside every table -> bypass escape
    sym[::89] = -7777
    data = O.GaussianTables.encode(tabs, sym, idx)
    assert len(data) % 4 == 0
    dec = tabs.decoder(data)
    out = np.concatenate([dec.decode_stream(idx[i:i + 96]) for i in range(0, 5000, 96)])
    assert np.array_equal(out, sym)


def test_layout_matches_reference():
    g = load_golden("loop_tiny_ks3111")
    img = g["image"].astype(np.float32) / 255.0 - 0.5
    xb = O.image_to_blocks(img, int(g["B"]))
    assert np.array_equal(xb, g["x"])
    assert np.array_equal(O.blocks_to_image(xb, int(g["B"])), img)


def test_stages_b8_lowrate():
    """Teacher-forced per-stage activations of compress_blk at full B8_lowrate width."""
    g = load_golden("stages_b8_lowrate")
    from lbic.arch import Arch
    arch = Arch(8, (3, 1, 1, 1), 768, 96)
    net = O.OracleNet(arch, synth_state_dict(arch, 1337))
    loop = load_golden("loop_b8_lowrate_2rows")
    table = O.scale_table()
    for bi, (v, h) in enumerate(g["blocks"]):
        win = np.transpose(g["win"][bi], (1, 2, 0))          # [3,3,C]
        ksi = net.ctx(win)
        assert _close(ksi, g["ksi"][bi]) < RTOL
        scales, means = g["ksi"][bi][:96], g["ksi"][bi][96:]
        y = net.fwd(win, loop["x"][v, h])
        assert _close(y, g["y"][bi]) < RTOL
        assert np.array_equal(O.build_indexes(scales, table), g["idx"][bi])
        sym = np.rint(y - means).astype(np.int32)
        assert np.array_equal(sym, g["sym"][bi])
        xhat = net.inv(win, g["yq"][bi])
        assert _close(xhat, g["xhat"][bi]) < RTOL
        bits = O.likelihood_bits(g["yq"][bi], scales, means)
        assert _close(bits, g["bits"][bi]) < 1e-4


LOOPS = ["tiny_ks3111", "tiny_ks3311", "b4_highrate", "b16_lowrate", "b8_highrate", "b8_lowrate_2rows",
         "b8_highrate_mid", "b4_highrate_mid", "b16_lowrate_low"]


@pytest.mark.parametrize("name", LOOPS)
def test_closed_loop_matches_reference(name):
    """The raster closed loop (compress) reproduces the reference's symbols / indexes bit-exactly and its
    reconstruction within 1e-5; decompress() of our own bitstream reproduces the reference decoder."""
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    codec = O.OracleCodec(arch, synth_state_dict(arch, int(g["weight_seed"]), rate=golden_rate(g)))
    out = codec.compress(g["x"])
    assert np.array_equal(out["indexes"], g["indexes"])
    assert np.array_equal(out["symbols"], g["symbols"])
    assert np.abs(out["zhat"] - g["zhat"]).max() < 1e-5
    assert np.array_equal(g["zhat"], g["zhat_dec"])          # the reference's own enc/dec agreement
    if name in ("tiny_ks3111", "tiny_ks3311"):
        zdec = codec.decompress(out["bytes"], *g["x"].shape[:2])
        assert np.array_equal(zdec, out["zhat"])


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
def test_oracle_forward_matches_reference(name):
    """The oracle's teacher-forced full-frame forward (net:90-106) against the reference's forward() fixture:
    xhat within 1e-5, self-information within 1e-4 relative (fp32 erfc)."""
    g = load_golden("forward_" + name)
    arch = golden_arch(g)
    net = O.OracleNet(arch, synth_state_dict(arch, int(g["weight_seed"])))
    xhat, info = net.forward_frame(g["zhat"], g["x"])
    assert np.abs(xhat - g["xhat"]).max() < 1e-5
    assert (np.abs(info - g["self_info"]) <= 1e-4 * np.maximum(1.0, np.abs(g["self_info"]))).all()


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
def test_oracle_validate_recu_matches_reference(name):
    """validate_recu_reco_fast (agent:491-520) semantics: the oracle's closed loop with forward()'s border
    rule against the reference's loop around its own forward()."""
    g = load_golden("recu_" + name)
    arch = golden_arch(g)
    codec = O.OracleCodec(arch, synth_state_dict(arch, int(g["weight_seed"])))
    z, info = codec.validate_recu(g["x"])
    assert np.abs(z - g["zhat"]).max() < 1e-5
    assert (np.abs(info - g["self_info"]) <= 1e-4 * np.maximum(1.0, np.abs(g["self_info"]))).all()


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
def test_torch_cpu_restatement_matches_reference(name):
    """oracle/torch_ref.py (bench.py's CPU baseline) reproduces the reference's closed loop bit-exactly on the
    tie-screened fixtures, and its decoder inverts its encoder."""
    import torch
    from oracle.torch_ref import TorchRef
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    torch.set_num_threads(1)
    t = TorchRef(arch, synth_state_dict(arch, int(g["weight_seed"])))
    r = t.compress(g["x"])
    assert np.array_equal(r["symbols"], g["symbols"])
    assert np.array_equal(r["indexes"], g["indexes"])
    assert np.abs(r["zhat"] - g["zhat"]).max() < 1e-5
    assert np.array_equal(t.decompress(r["bytes"], *g["x"].shape[:2]), r["zhat"])
