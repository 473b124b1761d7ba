"""The single-image decoder (k_dec_one, csrc/one.hip): lbc_decode of ONE image -- the reference's own per-image path,
decompress() (graphs/models/BlockBasedImgCompLossy_net.py:400-452) as eval_model calls it
(agents/blkbsdimgcomp_agent.py:591-599) -- as one persistent launch with every weight tile resident in LDS.

* The reference's stream of every KS3111 closed-loop fixture (re-made by the oracle coder from the fixture's symbols and
  indexes) decoded by k_dec_one equals the fixture's ``zhat_dec`` (the reference's decompress()) within 1e-5 relative,
  and equals the row-graph decoder (LBIC_ONE=0) bit for bit.
* Library-encoded frames of ragged shapes (one block row, one block column, two columns, odd sizes) decode bit-exactly
  to the encoder's reconstruction, through k_dec_one.
* The full 768x768 B8_lowrate frame: tests/test_fullsize_gpu.py::test_full_frame_b8_lowrate_vs_reference decodes it as
  one image through k_dec_one (asserted there: ``decode_path()`` and no timeout).
* A launch whose waits time out (LBIC_ONE_TMO=1 tick) is decoded by the row graphs instead, counted, same result.
* Truncated and corrupted streams decoded through k_dec_one raise (an overrun, or a decode that does not end in the
  encoder's initial rANS state), without a timeout, and the handle decodes correctly afterwards.
* KS[1] = 3 (round 6): the context net under the layer-0 cache, B4_highrate's K = 3,840 layer 1 held as half tiles by
  two workgroups, the high-rate streams through the sparse coder's table search -- the reference's own streams of the
  KS3311 fixtures (tiny, B4_highrate at both operating points) and ragged B4 frames (one block column: three positions
  in layer 0's MFMA at every step) decode through k_dec_one, equal the reference's decompress() and the row graphs bit
  for bit; a damaged B4 stream raises.
* Several images keep the row graphs; weights past the grid's LDS (B8_highrate, B16_lowrate) too.
"""
import types

import numpy as np
import pytest
import torch

from conftest import assert_rel, golden_arch, golden_rate, load_golden
from lbic.weights import synth_state_dict
from oracle import oracle as O

pytestmark = pytest.mark.gpu

_M = {}


def _model(arch, seed, rate):
    from lbic.model import BlockBasedImgCompLossyNetv9
    key = (arch, seed, rate)
    if key not in _M:
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, seed, rate=rate))
        m.update(force=True)
        _M[key] = m
    return _M[key]


@pytest.mark.parametrize("name", ["tiny_ks3111", "b8_lowrate_2rows", "b16_lowrate", "b16_lowrate_low", "tiny_ks3311",
                                  "b4_highrate_mid", "b4_highrate", "b8_highrate_mid"])
def test_one_decodes_reference_stream(name, monkeypatch):
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")       # k_dec_one decodes with the sparse rANS variant (any rate)
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    Hb, Wb = g["x"].shape[:2]
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    m = _model(arch, int(g["weight_seed"]), golden_rate(g))
    z1 = m.decompress_batch([stream], Hb, Wb)
    path = m.decode_path()
    monkeypatch.setenv("LBIC_ONE", "0")
    zg = m.decompress_batch([stream], Hb, Wb)
    assert m.decode_path()["path"] == "graphs"
    ref = g["zhat_dec"]
    assert_rel(z1[0].cpu().numpy(), ref, what=f"{name}: single-image decode vs the reference's decompress()")
    assert torch.equal(z1, zg), f"{name}: k_dec_one != row graphs ({(z1 != zg).sum().item()} values)"
    print(f"{name} (N{arch.N} B{arch.B}, {Hb}x{Wb} blocks): path {path['path']}, "
          f"max |zhat - zhat_dec(ref)| = {float(np.abs(z1[0].cpu().numpy() - ref).max()):.3e}")
    if name in ("tiny_ks3111", "b8_lowrate_2rows", "tiny_ks3311", "b4_highrate_mid", "b4_highrate"):
        assert path["path"] == "one", path
        assert path["one_timeouts"] == 0, path


@pytest.mark.parametrize("Hb,Wb", [(1, 7), (5, 1), (3, 2), (4, 9), (2, 96)])
def test_one_roundtrip_ragged(Hb, Wb):
    from lbic.arch import Arch
    arch = Arch(8, (3, 1, 1, 1), 768, 96)
    m = _model(arch, 1337, "low")
    x = torch.from_numpy(np.random.default_rng(Hb * 100 + Wb).integers(0, 256, (1, Hb, Wb, arch.cx))
                         .astype(np.float32) / 255.0 - 0.5).cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    z = m.decompress_batch(st, Hb, Wb)
    assert m.decode_path()["path"] == "one"
    assert torch.equal(z, r["zhat"]), f"{Hb}x{Wb}: decode != encode"


@pytest.mark.parametrize("Hb,Wb", [(1, 5), (4, 1), (3, 2), (3, 7)])
def test_one_roundtrip_ragged_ks3311(Hb, Wb):
    """B4_highrate (KS3311, layer-0 cache, half-tile layer 1) at its mid operating point: ragged frames -- one block row,
    one block column (row ends on both sides at every step: three layer-0 positions), two columns -- decode through
    k_dec_one to the encoder's reconstruction bit for bit."""
    from lbic.arch import Arch
    arch = Arch(4, (3, 3, 1, 1), 512, 96)
    m = _model(arch, 1337, "mid")
    x = torch.from_numpy(np.random.default_rng(Hb * 100 + Wb).integers(0, 256, (1, Hb, Wb, arch.cx))
                         .astype(np.float32) / 255.0 - 0.5).cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    z = m.decompress_batch(st, Hb, Wb)
    p = m.decode_path()
    assert p["path"] == "one" and p["one_timeouts"] == 0, p
    assert torch.equal(z, r["zhat"]), f"{Hb}x{Wb}: decode != encode ({(z != r['zhat']).sum().item()} values)"


def test_one_timeout_falls_back(monkeypatch):
    from lbic.arch import Arch
    arch = Arch(8, (3, 1, 1, 1), 768, 96)
    m = _model(arch, 1337, "low")
    x = torch.from_numpy(np.random.default_rng(5).integers(0, 256, (1, 3, 4, arch.cx))
                         .astype(np.float32) / 255.0 - 0.5).cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    t0 = m.decode_path()["one_timeouts"]
    monkeypatch.setenv("LBIC_ONE_TMO", "1")
    z = m.decompress_batch(st, 3, 4)
    p = m.decode_path()
    assert p["path"] == "graphs" and p["one_timeouts"] == t0 + 1, p
    assert torch.equal(z, r["zhat"])
    monkeypatch.delenv("LBIC_ONE_TMO")
    z = m.decompress_batch(st, 3, 4)
    assert m.decode_path()["path"] == "one"
    assert torch.equal(z, r["zhat"])


def test_one_not_for_batches():
    g = load_golden("loop_tiny_ks3111")
    arch = golden_arch(g)
    m = _model(arch, int(g["weight_seed"]), golden_rate(g))
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    Hb, Wb = g["x"].shape[:2]
    z = m.decompress_batch([stream, stream], Hb, Wb)
    assert m.decode_path()["path"] == "graphs"            # two images: the row graphs
    assert torch.equal(z[0], z[1])


@pytest.mark.parametrize("damage", ["truncated", "corrupt_head", "corrupt_tail"])
@pytest.mark.parametrize("name", ["tiny_ks3111", "b4_highrate_mid"])
def test_one_bad_stream_raises(damage, name, monkeypatch):
    """A damaged stream through k_dec_one (sparse rANS forced, so the low-rate kernel runs whatever the stream's rate):
    the decode raises instead of returning a wrong image, no wait times out, and the handle still decodes."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    Hb, Wb = g["x"].shape[:2]
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    m = _model(arch, int(g["weight_seed"]), golden_rate(g))
    good = m.decompress_batch([stream], Hb, Wb)
    assert m.decode_path()["path"] == "one"
    w = bytearray(stream)
    if damage == "truncated":
        w = w[:len(w) // 2 - (len(w) // 2) % 4]
    elif damage == "corrupt_head":                  # the initial coder state
        w[0:4] = bytes(b ^ 0x5A for b in w[0:4])
    else:                                           # a word the last blocks read
        w[-4:] = bytes(b ^ 0xA5 for b in w[-4:])
    t0 = m.decode_path()["one_timeouts"]
    with pytest.raises((RuntimeError, ValueError)):
        m.decompress_batch([bytes(w)], Hb, Wb)
    p = m.decode_path()
    assert p["path"] == "one" and p["one_timeouts"] == t0, p
    assert torch.equal(m.decompress_batch([stream], Hb, Wb), good)
    assert m.decode_path()["path"] == "one"


@pytest.mark.parametrize("path", ["one", "graphs", "team"])
def test_trailing_padding_words_ignored(path, monkeypatch):
    """Words after the last one a decode reads are ignored, as CompressAI's RansDecoder ignores them: a
    reference-format stream with trailing zero words decodes to the same image through k_dec_one, the row graphs and a
    team launch, while a corrupted last word still raises (the end-state check, lbic.h lbc_decode)."""
    from lbic.model import decompress_teams
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    g = load_golden("loop_tiny_ks3111")
    arch = golden_arch(g)
    Hb, Wb = g["x"].shape[:2]
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    m = _model(arch, int(g["weight_seed"]), golden_rate(g))
    padded = stream + bytes(8)
    bad = bytearray(padded)
    bad[len(stream) - 4:len(stream)] = bytes(b ^ 0xA5 for b in bad[len(stream) - 4:len(stream)])
    if path == "team":
        hs = [m, m.sibling()]
        good = decompress_teams(hs, [[stream] * 2] * 2, Hb, Wb)
        got = decompress_teams(hs, [[padded] * 2] * 2, Hb, Wb)
        assert hs[0].team_stats()["mode"] == "team_sparse"
        assert all(torch.equal(a, b) for a, b in zip(got, good))
        with pytest.raises((RuntimeError, ValueError)):
            decompress_teams(hs, [[padded, bytes(bad)]] * 2, Hb, Wb)
        return
    n = 1 if path == "one" else 2
    good = m.decompress_batch([stream] * n, Hb, Wb)
    assert torch.equal(m.decompress_batch([padded] * n, Hb, Wb), good)
    assert m.decode_path()["path"] == path
    assert_rel(good[0].cpu().numpy(), g["zhat_dec"], what="decoded zhat vs the reference's decompress()")
    with pytest.raises((RuntimeError, ValueError)):
        m.decompress_batch([bytes(bad)] * n, Hb, Wb)
