"""The headline decoder (lbc_decode_team / k_dec_team) against the reference's OWN decompress() output.

* Every closed-loop fixture (tests/golden/loop_*.npz) holds ``zhat_dec``: the reconstruction the reference's
  decompress() (graphs/models/BlockBasedImgCompLossy_net.py:400-452) produced from the reference's stream of the
  fixture's symbols.  That stream is re-made here by the oracle coder (oracle/rans_oracle.c, byte-identical to the
  product coder: tests/test_gpu_parity.py) from the fixture's symbols and indexes, and decoded by team launches --
  copies of it in every image slot of several teams, both team geometries (one XCD slot per team, and teams of two
  XCD slots with write-through hand-offs) and both rANS variants.  Every decoded image must equal ``zhat_dec`` within 1e-5
  relative (north_star's bar) and be bit-identical across copies.
* The full 768x768 B8_lowrate frame (frame_b8_lowrate.npz, the reference's compress() closed loop) inside a launch of
  the headline's shape: 8 teams x 32 frames of 768x768.  Team t carries the fixture's stream in image slot t and 31
  other frames (encoded by the library) around it.  The fixture image must match the reference's reconstruction rows
  and per-block sums within 1e-5 relative, every other image the encoder's reconstruction bit for bit.  The stream
  codes the fixture's symbols with the scale indexes this library derives (equal to the reference's everywhere except
  at the fixture's listed near ties, asserted): the decoder derives those same indexes, so at a near-tie flip the
  reference's own bytes would not decode here, while the symbols -- and so the reconstruction -- are the reference's.
"""
import hashlib
import types

import numpy as np
import pytest
import torch

from conftest import assert_rel, golden_arch, golden_rate, load_golden
from lbic.weights import synth_state_dict
from oracle import oracle as O

pytestmark = pytest.mark.gpu

LOOPS = ["tiny_ks3111", "tiny_ks3311", "b4_highrate", "b16_lowrate", "b8_highrate", "b8_lowrate_2rows",
         "b8_highrate_mid", "b4_highrate_mid", "b16_lowrate_low"]
_H = {}


def _handles(arch, seed, rate, T):
    from lbic.model import BlockBasedImgCompLossyNetv9
    key = (arch, seed, rate)
    if key not in _H:
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, seed, rate=rate))
        m.update(force=True)
        _H[key] = [m]
    hs = _H[key]
    while len(hs) < T:
        hs.append(hs[0].sibling())
    return hs[:T]


@pytest.mark.parametrize("spread", [1, 2])
@pytest.mark.parametrize("sparse", ["0", "1"])
@pytest.mark.parametrize("name", LOOPS)
def test_team_decodes_reference_stream(name, sparse, spread, monkeypatch):
    from lbic.model import decompress_teams
    monkeypatch.setenv("LBIC_RANS_SPARSE", sparse)
    monkeypatch.setenv("LBIC_TEAM_SPREAD", str(spread))
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    Hb, Wb = g["x"].shape[:2]
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    T, n = 3, 2
    hs = _handles(arch, int(g["weight_seed"]), golden_rate(g), T)
    got = decompress_teams(hs, [[stream] * n for _ in range(T)], Hb, Wb)
    st = hs[0].team_stats()
    assert st["mode"] == ("team_sparse" if sparse == "1" else "team_dense"), st
    assert st["plain"] == (1 if spread == 1 else 0), st
    ref = g["zhat_dec"]
    worst = 0.0
    for t in range(T):
        for i in range(n):
            z = got[t][i].cpu().numpy()
            assert torch.equal(got[t][i], got[0][0]), f"team {t} image {i} differs from team 0 image 0"
            assert_rel(z, ref, what=f"team {t} image {i} vs the reference's decompress()")
            worst = max(worst, float(np.abs(z - ref).max()))
    print(f"{name} spread={spread} sparse={sparse}: max |zhat - zhat_dec(ref)| = {worst:.3e} (bar {1e-5 * np.abs(ref).max():.3e})")


@pytest.mark.parametrize("sparse", ["0", "1"])
@pytest.mark.parametrize("name,n", [("tiny_ks3311", 32), ("b4_highrate_mid", 32), ("b8_highrate_mid", 32),
                                    ("b16_lowrate_low", 32), ("b8_lowrate_2rows", 32),
                                    ("b8_highrate_mid", 6), ("b16_lowrate_low", 16)])
def test_team_reference_stream_headline_geometry(name, n, sparse, monkeypatch):
    """The headline's launch geometry -- 16 teams, two per XCD slot (sub = 2), each half an XCD's CUs -- on the
    reference's own stream at high rate, with the KS3311 layer-0 cache and at B16: n = 32 copies per team (one 32-frame
    batch per team, configs 2 and 4), n = 6 (config 3's HEAD default: two 3-frame Kodak shards per team) and n = 16
    (config 5's: two 8-frame batches per team).  Every image must equal the reference's decompress() output within
    1e-5 relative and every copy be bit-identical.  The dense coder may give way to the sparse one where its tables do
    not fit a workgroup's LDS beside the partials (bit-identical, lbc_decode_team); the row-graph fallback may not run."""
    from lbic.model import decompress_teams
    monkeypatch.setenv("LBIC_RANS_SPARSE", sparse)
    monkeypatch.delenv("LBIC_TEAM_SPREAD", raising=False)
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    Hb, Wb = g["x"].shape[:2]
    stream = O.GaussianTables().encode(g["symbols"], g["indexes"])
    T = 16
    hs = _handles(arch, int(g["weight_seed"]), golden_rate(g), T)
    got = decompress_teams(hs, [[stream] * n for _ in range(T)], Hb, Wb)
    st = hs[0].team_stats()
    assert st["mode"] in (("team_sparse",) if sparse == "1" else ("team_sparse", "team_dense")), st
    assert st["plain"] == 1 and st["timeout_fallbacks"] == 0, st
    ref = g["zhat_dec"]
    assert_rel(got[0][0].cpu().numpy(), ref, what=f"{name} T=16 n={n} vs the reference's decompress()")
    for t in range(T):
        assert got[t].shape[0] == n
        for i in range(n):
            assert torch.equal(got[t][i], got[0][0]), f"team {t} image {i} differs from team 0 image 0"
    print(f"{name} T=16 n={n} sparse={sparse} ({st['mode']}): max |zhat - zhat_dec(ref)| = "
          f"{float(np.abs(got[0][0].cpu().numpy() - ref).max()):.3e}")


def test_team_full_frame_in_headline_launch(monkeypatch):
    from lbic.layout import image_to_blocks
    from lbic.model import decompress_teams
    monkeypatch.delenv("LBIC_RANS_SPARSE", raising=False)
    g = load_golden("frame_b8_lowrate")
    arch = golden_arch(g)
    H, W = int(g["H"]), int(g["W"])
    Hb, Wb = H // arch.B, W // arch.B
    img = np.random.default_rng(int(g["image_seed"])).integers(0, 256, (1, 3, H, W), dtype=np.uint8)[0]
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["image_sha256"])
    T, n = 16, 32          # the headline's launch: 16 batches of 32 frames, two teams per XCD
    hs = _handles(arch, int(g["weight_seed"]), str(g["rate"]), T)
    m = hs[0]
    xb = torch.from_numpy(image_to_blocks(img.astype(np.float32) / 255.0 - 0.5, arch.B))[None].cuda()
    r = m.compress_batch(xb)
    sym, idx = r["symbols"][0].cpu().numpy(), r["indexes"][0].cpu().numpy()
    ties = set(g["near_tie_symbols"].tolist()) | set(g["near_tie_indexes"].tolist())
    assert np.array_equal(sym, g["symbols"]), "symbols differ from the reference's closed loop"
    flips = np.nonzero(idx != g["indexes"].astype(np.int32))[0]
    assert all(int(i) in ties for i in flips), "scale-index flips off the fixture's near ties"
    fixture_stream = O.GaussianTables().encode(g["symbols"], idx)
    # 31 other frames, encoded by the library; team t gets them rotated by t with the fixture in slot t
    gen = torch.Generator(device="cuda").manual_seed(7)
    xo = torch.randint(0, 256, (n - 1, Hb, Wb, arch.cx), generator=gen, device="cuda", dtype=torch.uint8)
    ro = m.compress_batch(xo.float().div_(255.0).sub_(0.5))
    so = m.entropy_encode(ro["symbols"], ro["indexes"])
    batches, owners = [], []
    for t in range(T):
        order = [(k + t) % (n - 1) for k in range(n - 1)]
        b = [so[k] for k in order]
        b.insert(t, fixture_stream)
        batches.append(b)
        owners.append(order[:t] + [-1] + order[t:])
    got = decompress_teams(hs, batches, Hb, Wb)
    st = hs[0].team_stats()
    assert st["mode"] == "team_sparse", st
    rows, zr = g["zhat_rows"], g["zhat_row_data"]
    for t in range(T):
        for i, k in enumerate(owners[t]):
            if k >= 0:
                assert torch.equal(got[t][i], ro["zhat"][k]), f"team {t} image {i} != its encoder reconstruction"
        z = got[t][t].cpu().numpy()
        dz = float(np.abs(z[rows] - zr).max())
        dsum = float(np.abs(z.astype(np.float64).sum(-1) - g["zhat_block_sum"]).max())
        assert dz <= 1e-5 * float(np.abs(zr).max()), f"team {t}: zhat rows differ from the reference by {dz}"
        assert dsum <= 1e-5 * float(np.abs(z).sum(-1).max()), f"team {t}: block sums differ by {dsum}"
        assert torch.equal(got[t][t], r["zhat"][0])
    print(f"headline launch: fixture frame in {T} teams, max |dzhat| rows {dz:.3e}, block sums {dsum:.3e}, "
          f"{len(flips)} scale-index flips at listed near ties")
