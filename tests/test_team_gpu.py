"""Team decoder (lbc_decode_team / k_dec_team): several batches decoded by ONE persistent launch, one team of
workgroups per batch, must reproduce the graph decoder (lbc_decode, itself bit-exact against the encoder and the
reference's closed loops in test_gpu_parity.py) bit for bit: every geometry class of the recorded raster step
(KS3111, KS3311 with the layer-0 cache's border classes), ragged frames, image counts that do not fill a 16-row
tile or need three row tiles, tiny teams (many output tiles per workgroup: the weight-prefetch loop), corrupt
streams, both rANS variants (sparse at low rates, dense with the tables in LDS at high rates), and the fallback."""
import types

import numpy as np
import pytest
import torch

from conftest import golden_arch, load_golden
from lbic.weights import synth_state_dict

pytestmark = pytest.mark.gpu

_M = {}


def handles(name, T):
    """T sibling handles (one per batch) of the fixture's architecture and weights."""
    from lbic.model import BlockBasedImgCompLossyNetv9
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    if name not in _M:
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, int(g["weight_seed"])))
        m.update(force=True)
        _M[name] = [m]
    hs = _M[name]
    while len(hs) < T:
        hs.append(hs[0].sibling())
    return arch, hs[:T]


def batches(arch, T, n, Hb, Wb, seed, scale=0.5):
    rng = np.random.default_rng(seed)
    return [torch.from_numpy((rng.random((n, Hb, Wb, arch.cx), dtype=np.float32) - 0.5) * scale * 2).cuda()
            for _ in range(T)]


def run_case(name, T, n, Hb, Wb, seed=0, scale=0.05, wpc=1):
    """Encode T batches, decode them by the graph decoder and by one team launch; return both."""
    from lbic.model import decompress_teams
    arch, hs = handles(name, T)
    xs = batches(arch, T, n, Hb, Wb, seed, scale)
    rs = [hs[0].compress_batch(x) for x in xs]
    st = [hs[0].entropy_encode(r["symbols"], r["indexes"]) for r in rs]
    ref = [hs[0].decompress_batch(s, Hb, Wb) for s in st]
    for r, z in zip(rs, ref):
        assert torch.equal(r["zhat"], z)
    got = decompress_teams(hs, st, Hb, Wb, wg_per_cu=wpc)
    return ref, got, hs, st


@pytest.mark.parametrize("name,T,n,shape", [
    ("tiny_ks3111", 1, 4, None), ("tiny_ks3111", 3, 5, None), ("tiny_ks3311", 8, 3, None),
    ("b8_lowrate_2rows", 8, 32, (2, 96)), ("b8_lowrate_2rows", 2, 40, (2, 20)), ("b8_lowrate_2rows", 5, 48, (2, 9)),
    ("b8_lowrate_2rows", 8, 64, (2, 5)), ("b8_lowrate_2rows", 3, 50, (2, 6)), ("b8_lowrate_2rows", 2, 96, (2, 4)),
    ("b8_lowrate_2rows", 16, 32, (2, 6)), ("tiny_ks3311", 12, 3, None), ("b8_lowrate_2rows", 9, 40, (2, 5)),
])
def test_team_equals_graph_decoder(name, T, n, shape, monkeypatch):
    """Image counts of one to six row tiles, 1-16 teams (9-16: two teams per XCD, each half its CUs; 12 and 9: XCD
    slots with one team and with two).  64 images on a team of 32 workgroups (the bench's two-batch
    teams): up to 9 output tiles per workgroup on the fast path and two rANS waves per workgroup, each keeping its
    image's coder state in LDS; 50: some workgroups with one image; 96: three images per workgroup (each rANS wave
    decodes its rows one after another) and six row tiles (the long GEMM path)."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")     # the team kernel decodes with the sparse rANS variant
    g = load_golden("loop_" + name)
    Hb, Wb = shape or g["x"].shape[:2]
    ref, got, hs, _ = run_case(name, T, n, Hb, Wb, seed=T * 7 + n)
    for t in range(T):
        assert torch.equal(got[t], ref[t]), f"team {t}: {(got[t] != ref[t]).sum().item()} values differ"
    st = hs[0].team_stats()
    assert st["mode"] == "team_sparse", st


@pytest.mark.parametrize("name,T,n,shape", [("tiny_ks3311", 3, 5, (3, 4)), ("b8_lowrate_2rows", 4, 32, (2, 24))])
def test_team_write_through_mode(name, T, n, shape, monkeypatch):
    """LBIC_TEAM_SC1=1: every hand-off written through (k_dec_team<false>, the form that does not need a team's
    workgroups on one XCD; the default launch reruns in it when the placement census finds a team spread out)."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    monkeypatch.setenv("LBIC_TEAM_SC1", "1")
    ref, got, _, _ = run_case(name, T, n, *shape, seed=11)
    for t in range(T):
        assert torch.equal(got[t], ref[t])


@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (7, 1), (3, 5), (2, 2)])
def test_team_ragged_frames_ks3311(shape, monkeypatch):
    """One block, one row, one column, odd rectangles: the three column classes of the KS3311 step (layer-0 cache
    border cells at h = 0 and h = Wb - 1, both at once when Wb = 1)."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    ref, got, _, _ = run_case("tiny_ks3311", 3, 2, *shape, seed=sum(shape))
    for t in range(3):
        assert torch.equal(got[t], ref[t])


@pytest.mark.parametrize("name,T,n,shape", [("b8_lowrate_2rows", 8, 32, (2, 96)), ("tiny_ks3311", 8, 3, None),
                                            ("b8_lowrate_2rows", 3, 35, (2, 7))])
def test_team_two_workgroups_per_cu(name, T, n, shape, monkeypatch):
    """LBC_OPT_TEAM_WG_PER_CU = 2 (the launch with the GPU otherwise idle): teams of twice the workgroups, two per
    CU, each workgroup half the output tiles -- the same results; then a one-per-CU launch on the same handles."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    g = load_golden("loop_" + name)
    Hb, Wb = shape or g["x"].shape[:2]
    ref, got, hs, st = run_case(name, T, n, Hb, Wb, seed=T + n, wpc=2)
    for t in range(T):
        assert torch.equal(got[t], ref[t]), f"team {t}: {(got[t] != ref[t]).sum().item()} values differ"
    from lbic.model import decompress_teams
    got = decompress_teams(hs, st, Hb, Wb, wg_per_cu=1)
    for t in range(T):
        assert torch.equal(got[t], ref[t])


@pytest.mark.parametrize("spread", [1, 2])
@pytest.mark.parametrize("name,T,n,shape", [("b8_lowrate_2rows", 4, 32, (2, 24)), ("tiny_ks3311", 3, 5, (3, 4)),
                                            ("b8_lowrate_2rows", 1, 35, (2, 7)), ("b8_lowrate_2rows", 2, 64, (2, 6))])
def test_team_spread_two_xcds(name, T, n, shape, spread, monkeypatch):
    """At most four batches: by default each team takes the workgroups of two XCD slots (twice the ranks,
    write-through hand-offs); LBIC_TEAM_SPREAD=1 keeps one XCD per team (plain hand-offs) -- the same results as the
    graph decoder either way."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    monkeypatch.setenv("LBIC_TEAM_SPREAD", str(spread))
    ref, got, hs, _ = run_case(name, T, n, *shape, seed=T + 2 * n)
    for t in range(T):
        assert torch.equal(got[t], ref[t]), f"team {t}: {(got[t] != ref[t]).sum().item()} values differ"
    st = hs[0].team_stats()
    assert st["mode"] == "team_sparse" and st["plain"] == (0 if spread == 2 else 1)


@pytest.mark.parametrize("S", [1, 3, 7])
def test_team_small_teams(S, monkeypatch):
    """Teams of 1, 3 and 7 workgroups (LBC_OPT_TEAM_SIZE): every workgroup walks many output tiles per GEMM (the
    weight-prefetch loop, row tiles changing between items) and decodes several rANS streams per step."""
    from lbic.model import decompress_teams
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    monkeypatch.setenv("LBIC_TEAM_SPREAD", "1")
    ref, _, hs, st = run_case("b8_lowrate_2rows", 2, 35, 2, 6, seed=S)
    got = decompress_teams(hs, st, 2, 6, team_size=S)
    for t in range(2):
        assert torch.equal(got[t], ref[t])


@pytest.mark.parametrize("name,T,n,shape,scale", [
    ("tiny_ks3111", 3, 5, None, 0.05), ("tiny_ks3311", 8, 3, None, 0.05), ("b8_lowrate_2rows", 4, 32, (2, 24), 0.05),
    ("b8_lowrate_2rows", 2, 35, (2, 7), 4.0), ("tiny_ks3311", 3, 4, (3, 5), 4.0),
    ("b8_lowrate_2rows", 2, 64, (2, 7), 0.05)])
def test_team_dense_rans(name, T, n, shape, scale, monkeypatch):
    """The dense rANS variant inside the team kernel (high rates; every workgroup stages the tables in its LDS once per
    launch, one wave per stream runs rans_row<true>): forced by LBIC_RANS_SPARSE=0 at the fixtures' low rates, and
    picked by rate (>= 1 bit per symbol, bypass escapes included) on high-amplitude batches."""
    if scale < 1:
        monkeypatch.setenv("LBIC_RANS_SPARSE", "0")
    else:
        monkeypatch.delenv("LBIC_RANS_SPARSE", raising=False)
    g = load_golden("loop_" + name)
    Hb, Wb = shape or g["x"].shape[:2]
    ref, got, hs, st = run_case(name, T, n, Hb, Wb, seed=T * 5 + n, scale=scale)
    nsym = T * n * Hb * Wb * golden_arch(g).M
    for t in range(T):
        assert torch.equal(got[t], ref[t]), f"team {t}: {(got[t] != ref[t]).sum().item()} values differ"
    if scale >= 1:
        bits = 8.0 * sum(len(s) for b in st for s in b)
        assert bits / nsym >= 1.0, f"high-amplitude batch coded at {bits / nsym:.3f} bits per symbol"
    assert hs[0].team_stats()["mode"] == "team_dense"


def test_team_sparse_coder_at_high_rate(monkeypatch):
    """The sparse coder (tables in global memory) at more than one bit per symbol with two rANS waves per workgroup
    (64 images on a team of 32): what lbc_decode_team runs when the dense tables do not fit the workgroup's LDS beside
    the geometry's partials -- bit-identical to the graph decoder."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    ref, got, hs, st = run_case("b8_lowrate_2rows", 2, 64, 2, 5, seed=3, scale=4.0)
    nsym = 2 * 64 * 2 * 5 * 96
    assert 8.0 * sum(len(s) for b in st for s in b) / nsym >= 1.0
    for t in range(2):
        assert torch.equal(got[t], ref[t]), f"team {t}: {(got[t] != ref[t]).sum().item()} values differ"
    assert hs[0].team_stats()["mode"] == "team_sparse"


def test_team_fallback_and_errors(monkeypatch):
    """LBIC_TEAM=0: the batches decode through lbc_decode one after another with the same results; a truncated stream
    raises; the handles work afterwards."""
    from lbic.model import decompress_teams
    monkeypatch.setenv("LBIC_TEAM", "0")
    ref, got, hs, st = run_case("tiny_ks3111", 2, 3, 4, 5, seed=3)
    for t in range(2):
        assert torch.equal(got[t], ref[t])
    assert hs[0].team_stats()["mode"] == "fallback"
    monkeypatch.delenv("LBIC_TEAM")
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    bad = [list(st[0]), list(st[1])]
    bad[1][2] = bad[1][2][:8]
    with pytest.raises((ValueError, RuntimeError)):
        decompress_teams(hs, bad, 4, 5)
    with pytest.raises((ValueError, RuntimeError)):
        decompress_teams([hs[0], hs[0]], st, 4, 5)     # one handle twice
    got = decompress_teams(hs, st, 4, 5)
    for t in range(2):
        assert torch.equal(got[t], ref[t])
    assert hs[0].team_stats()["mode"] == "team_sparse"


def test_team_stamps(monkeypatch):
    """LBIC_TEAM_STAMPS=1 records the sampled step's barrier times and the launch span per team."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    monkeypatch.setenv("LBIC_TEAM_STAMPS", "1")
    _, _, hs, _ = run_case("tiny_ks3111", 2, 4, 4, 6, seed=5)
    ts = hs[0].team_stamps()
    assert len(ts) == 2
    for row in ts:
        assert row[63] > row[62] > 0 and row[61] > row[60] > 0


def test_team_barrier_timeout_falls_back(monkeypatch):
    """A team barrier that times out (forced: LBIC_TEAM_TMO=1 tick) ends the launch on every workgroup; the batches are
    then decoded through lbc_decode one after another in the same call, with the same results, and the event is
    counted (lbc_team_events) instead of failing the decode."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1")
    _, hs0 = handles("b8_lowrate_2rows", 1)
    before = hs0[0].team_stats()["timeout_fallbacks"]
    monkeypatch.setenv("LBIC_TEAM_TMO", "1")
    ref, got, hs, streams = run_case("b8_lowrate_2rows", 4, 32, 2, 12, seed=9)
    for t in range(4):
        assert torch.equal(got[t], ref[t])
    st = hs[0].team_stats()
    assert st["mode"] == "fallback" and st["timeout_fallbacks"] == before + 1, st
    monkeypatch.delenv("LBIC_TEAM_TMO")
    from lbic.model import decompress_teams
    got = decompress_teams(hs, streams, 2, 12)
    for t in range(4):
        assert torch.equal(got[t], ref[t])
    assert hs[0].team_stats()["mode"] == "team_sparse"


def test_team_dense_two_workgroups_per_cu(monkeypatch):
    """High rates (dense rANS, the ~70 KB table image in every workgroup's LDS) with LBC_OPT_TEAM_WG_PER_CU = 2: two
    such workgroups do not fit one CU's LDS, so the launch must shrink to one per CU (occupancy query on the dense
    instance with the launch's dynamic LDS) rather than start a grid that cannot be co-resident."""
    monkeypatch.delenv("LBIC_RANS_SPARSE", raising=False)
    _, hs0 = handles("b8_lowrate_2rows", 1)
    before = hs0[0].team_stats()["timeout_fallbacks"]      # (a per-handle counter: earlier tests may have counted)
    ref, got, hs, _ = run_case("b8_lowrate_2rows", 8, 32, 2, 7, seed=21, scale=4.0, wpc=2)
    for t in range(8):
        assert torch.equal(got[t], ref[t])
    st = hs[0].team_stats()
    assert st["mode"] == "team_dense" and st["timeout_fallbacks"] == before, st
