"""GPU parity: the HIP path (liblbic.so through the C ABI) against the reference golden vectors and the
oracle.  Bars: symbols and scale indexes bit-exact (tie-screened fixtures), reconstructions within
1e-5 relative (max |dz| <= 1e-5 max |z_ref|), bitstream bytes identical to the oracle coder on the same
symbols, decode(encode) bit-exact, estimated bits within 1e-4 relative of the oracle likelihood."""
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
_MODELS = {}


def model_for(arch, seed=1337, rate="high"):
    from lbic.model import BlockBasedImgCompLossyNetv9
    key = (arch, seed, rate)
    if key not in _MODELS:
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, seed, rate=rate))
        m.update(force=True)
        _MODELS[key] = m
    return _MODELS[key]


@pytest.fixture(scope="module")
def tables():
    return O.GaussianTables()


@pytest.mark.parametrize("name", LOOPS)
def test_closed_loop_matches_reference(name, tables):
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]), golden_rate(g))
    x = torch.from_numpy(g["x"])[None].cuda()
    r = m.compress_batch(x, want_bits=True)
    sym = r["symbols"][0].cpu().numpy()
    idx = r["indexes"][0].cpu().numpy()
    assert np.array_equal(idx, g["indexes"]), f"{(idx != g['indexes']).sum()} index mismatches"
    assert np.array_equal(sym, g["symbols"]), f"{(sym != g['symbols']).sum()} symbol mismatches"
    z = r["zhat"][0].cpu().numpy()
    assert_rel(z, g["zhat"], what="zhat")
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    assert streams[0] == tables.encode(g["symbols"], g["indexes"])
    zdec = m.decompress_batch(streams, *g["x"].shape[:2])
    assert torch.equal(zdec, r["zhat"]), "decoder reconstruction differs from the encoder's"
    assert_rel(zdec.cpu().numpy()[0], g["zhat_dec"], what="decoded zhat vs the reference's decompress()")
    bps = 8.0 * len(streams[0]) / sym.size
    print(f"{name} ({golden_rate(g)}): {bps:.3f} bits/symbol, rANS variant "
          f"{'sparse' if bps < 1.0 else 'dense'}, max |zhat - ref| {np.abs(z - g['zhat']).max():.2e}")


def test_bits_match_oracle_likelihood():
    g = load_golden("stages_b8_lowrate")
    loop = load_golden("loop_b8_lowrate_2rows")
    arch = golden_arch(loop)
    m = model_for(arch)
    r = m.compress_batch(torch.from_numpy(loop["x"])[None].cuda(), want_bits=True)
    bits = r["bits"][0].cpu().numpy().reshape(loop["x"].shape[0], loop["x"].shape[1], arch.M)
    for bi, (v, h) in enumerate(g["blocks"]):
        ref = g["bits"][bi]
        assert np.abs(bits[v, h] - ref).max() <= 1e-4 * max(1.0, np.abs(ref).max())


def test_batch_equals_single():
    """Images coded together (one wavefront over the batch) give bit-identical results to one at a time."""
    g = load_golden("loop_tiny_ks3311")
    arch = golden_arch(g)
    m = model_for(arch)
    rng = np.random.default_rng(5)
    imgs = [O.image_to_blocks(rng.integers(0, 256, (3, 32, 48)).astype(np.float32) / 255 - 0.5, 4) for _ in range(3)]
    xb = torch.from_numpy(np.stack(imgs)).cuda()
    rb = m.compress_batch(xb)
    for k in range(3):
        r1 = m.compress_batch(xb[k:k + 1].contiguous())
        assert torch.equal(r1["symbols"][0], rb["symbols"][k])
        assert torch.equal(r1["zhat"][0], rb["zhat"][k])
    streams = m.entropy_encode(rb["symbols"], rb["indexes"])
    assert torch.equal(m.decompress_batch(streams, 8, 12), rb["zhat"])


def test_reference_interface_roundtrip():
    """compress(x, LRU, chlat) / decompress(...) on the reference's NCHW block->channel tensors."""
    g = load_golden("loop_tiny_ks3111")
    arch = golden_arch(g)
    m = model_for(arch)
    x = torch.from_numpy(g["x"]).permute(2, 0, 1)[None].cuda()         # [1, 3B^2, Hb, Wb]
    lru = [arch.lru] * 3
    bs, zhat = m.compress(x, lru, arch.M)
    assert isinstance(bs, bytes) and len(bs) % 4 == 0
    zdec = m.decompress(bs, lru, x.shape, arch.M, x.device)
    assert torch.equal(zhat, zdec)
    assert_rel(zhat[0].permute(1, 2, 0).cpu().numpy(), g["zhat"], what="zhat")
    with pytest.raises(ValueError):
        m.compress(x, [arch.lru + 1] * 3, arch.M)


def test_uninitialized_cdf_raises():
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.arch import Arch
    arch = Arch(4, (3, 1, 1, 1), 64, 16)
    cfg = types.SimpleNamespace(block_size=4, KS=[3, 1, 1, 1], N=64, M=16, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, 1))
    with pytest.raises(ValueError, match="Run update"):
        m.compress_batch(torch.zeros(1, 2, 2, 48, device="cuda"))


def _teacher_forced_check(arch, xb, zhat, sym, idx, blocks):
    """Recompute sampled blocks on the CPU oracle given the GPU's own reconstruction (teacher forcing):
    symbols/indexes must agree wherever the oracle's rounding / table margins exceed 1e-4."""
    net = O.OracleNet(arch, synth_state_dict(arch, 1337))
    table = O.scale_table()
    L, M = arch.lru, arch.M
    Hb, Wb, C = xb.shape
    zp = np.zeros((Hb + 2 * L, Wb + 2 * L, C), np.float32)
    zp[L:L + Hb, L:L + Wb] = zhat
    checked = 0
    for (v, h) in blocks:
        win = zp[v:v + 2 * L + 1, h:h + 2 * L + 1].copy()
        win[L, L:] = 0
        win[L + 1:] = 0
        ksi = net.ctx(win)
        y = net.fwd(win, xb[v, h])
        d = (y - ksi[M:]).astype(np.float64)
        ok = np.abs(np.abs(d - np.floor(d)) - 0.5) > 1e-4
        s_ref = np.rint(d).astype(np.int32)
        sl = slice((v * Wb + h) * M, (v * Wb + h + 1) * M)
        assert np.array_equal(sym[sl][ok], s_ref[ok])
        raw = ksi[:M].astype(np.float64)
        okx = np.min(np.abs(raw[:, None] - table[None, :]) / table[None, :], axis=1) > 1e-4
        assert np.array_equal(idx[sl][okx], O.build_indexes(ksi[:M], table)[okx])
        checked += 1
    return checked


def test_large_frame_b8_lowrate_roundtrip_and_teacher_forced():
    """B8_lowrate at 2 x 256x256: decode(encode) bit-exact; sampled blocks agree with the oracle."""
    from lbic.arch import Arch
    arch = Arch(8, (3, 1, 1, 1), 768, 96)
    m = model_for(arch)
    rng = np.random.default_rng(11)
    imgs = np.stack([O.image_to_blocks(rng.integers(0, 256, (3, 256, 256)).astype(np.float32) / 255 - 0.5, 8)
                     for _ in range(2)])
    xb = torch.from_numpy(imgs).cuda()
    r = m.compress_batch(xb)
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    assert torch.equal(m.decompress_batch(streams, 32, 32), r["zhat"])
    blocks = [(0, 0), (0, 31), (5, 7), (17, 30), (31, 0), (31, 31)]
    n = _teacher_forced_check(arch, imgs[1], r["zhat"][1].cpu().numpy(), r["symbols"][1].cpu().numpy(),
                              r["indexes"][1].cpu().numpy(), blocks)
    assert n == len(blocks)


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311", "b8_lowrate_2rows"])
def test_substream_format_roundtrip(name, tables):
    """Opt-in per-row sub-stream format: each row stream equals the oracle coder's stream of that row's
    symbols, and the wavefront decoder reproduces the encoder's reconstruction bit-exactly."""
    import struct
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    Hb, Wb = g["x"].shape[:2]
    x = torch.from_numpy(np.stack([g["x"], g["x"][:, ::-1].copy()])).cuda()     # 2 images
    r = m.compress_batch(x)
    cont = m.entropy_encode(r["symbols"], r["indexes"], fmt="rows", Hb=Hb, Wb=Wb)
    sym = r["symbols"].cpu().numpy()
    idx = r["indexes"].cpu().numpy()
    per = Wb * arch.M
    for k in range(2):
        magic, hb = struct.unpack_from("<II", cont[k], 0)
        assert hb == Hb
        sizes = struct.unpack_from(f"<{Hb}I", cont[k], 8)
        off = 8 + 4 * Hb
        for v in range(Hb):
            assert cont[k][off:off + sizes[v]] == tables.encode(sym[k, v * per:(v + 1) * per], idx[k, v * per:(v + 1) * per])
            off += sizes[v]
    z = m.decompress_batch(cont, Hb, Wb, fmt="rows")
    assert torch.equal(z, r["zhat"])
    if name == "b8_lowrate_2rows":
        assert np.array_equal(sym[0], g["symbols"])


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
def test_forward_matches_reference(name):
    """forward(zhat, x) (net:90-106, eval) on the GPU against the reference's own output on the same given
    zhat: xhat within 1e-5 relative, self-information within 1e-4 relative."""
    g = load_golden("forward_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    to = lambda a: torch.from_numpy(a).permute(2, 0, 1)[None].cuda()          # [Hb, Wb, C] -> [1, C, Hb, Wb]
    xhat, info = m.forward(to(g["zhat"]), to(g["x"]))
    assert xhat.shape == (1, arch.cx, 8, 8) and info.shape == (1, arch.M, 8, 8)
    xhat = xhat[0].permute(1, 2, 0).cpu().numpy()
    info = info[0].permute(1, 2, 0).cpu().numpy()
    assert_rel(xhat, g["xhat"], what="xhat")
    assert (np.abs(info - g["self_info"]) <= 1e-4 * np.maximum(1.0, np.abs(g["self_info"]))).all()


@pytest.mark.parametrize("name", ["tiny_ks3111", "b8_lowrate_2rows", "tiny_ks3311"])
def test_forward_on_closed_loop_reconstruction(name):
    """Teacher forcing on the closed loop's own zhat reproduces the closed loop: clamp(xhat) = zhat and the
    self-information equals the encoder's bits, bit for bit (same kernels, same slice order).  KS3311:
    the blocks whose context window lies inside the frame (the border differs by design: forward()
    zero-pads the layer-0 map, compress() evaluates it on the zero-padded zhat)."""
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    x = torch.from_numpy(g["x"])[None].cuda()
    r = m.compress_batch(x, want_bits=True)
    Hb, Wb = g["x"].shape[:2]
    xhat, info = m.forward(r["zhat"].permute(0, 3, 1, 2), x.permute(0, 3, 1, 2))
    zf = torch.clamp(xhat, -0.5, 0.5).permute(0, 2, 3, 1)
    bits = r["bits"].view(1, Hb, Wb, arch.M)
    inf = info.permute(0, 2, 3, 1)
    if arch.KS[1] == 3:
        sl = (slice(None), slice(1, Hb), slice(1, Wb - 1))
        zf, z0, bits, inf = zf[sl], r["zhat"][sl], bits[sl], inf[sl]
    else:
        z0 = r["zhat"]
    assert torch.equal(zf, z0)
    assert torch.equal(inf, bits)


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
@pytest.mark.parametrize("shape", [(1, 1), (1, 9), (7, 1), (3, 5)])
def test_ragged_frames_roundtrip(name, shape):
    """Frames of 1 block, one block row, one block column and a small odd rectangle: decode(encode) is bit
    exact (reference and sub-stream formats), the streams equal the oracle coder's bytes, and teacher forcing
    on the reconstruction reproduces it (KS3311: the blocks whose context lies inside the frame)."""
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    Hb, Wb = shape
    rng = np.random.default_rng(Hb * 100 + Wb)
    img = rng.integers(0, 256, (2, 3, Hb * arch.B, Wb * arch.B)).astype(np.float32) / 255 - 0.5
    x = torch.from_numpy(np.stack([O.image_to_blocks(i, arch.B) for i in img])).cuda()
    r = m.compress_batch(x, want_bits=True)
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    tabs = O.GaussianTables()
    for k in range(2):
        assert streams[k] == tabs.encode(r["symbols"][k].cpu().numpy(), r["indexes"][k].cpu().numpy())
    assert torch.equal(m.decompress_batch(streams, Hb, Wb), r["zhat"])
    rows = m.entropy_encode(r["symbols"], r["indexes"], fmt="rows", Hb=Hb, Wb=Wb)
    assert torch.equal(m.decompress_batch(rows, Hb, Wb, fmt="rows"), r["zhat"])
    xhat, info = m.forward(r["zhat"].permute(0, 3, 1, 2), x.permute(0, 3, 1, 2))
    zf = torch.clamp(xhat, -0.5, 0.5).permute(0, 2, 3, 1)
    inf = info.permute(0, 2, 3, 1)
    bits = r["bits"].view(2, Hb, Wb, arch.M)
    if arch.KS[1] == 3:
        sl = (slice(None), slice(1, Hb), slice(1, Wb - 1))
        zf, z0, inf, bits = zf[sl], r["zhat"][sl], inf[sl], bits[sl]
    else:
        z0 = r["zhat"]
    assert torch.equal(zf, z0) and torch.equal(inf, bits)


def test_bad_inputs_raise():
    """Errors are loud: empty batches, truncated / corrupted streams, a wrong container, wrong shapes."""
    g = load_golden("loop_tiny_ks3111")
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    x = torch.from_numpy(g["x"])[None].cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    Hb, Wb = g["x"].shape[:2]
    with pytest.raises((ValueError, RuntimeError)):
        m.compress_batch(x[:0])
    with pytest.raises((ValueError, RuntimeError)):
        m.decompress_batch([st[0][:8]], Hb, Wb)                    # truncated: the decoder runs out of words
    with pytest.raises((ValueError, RuntimeError)):
        m.decompress_batch([st[0][:5]], Hb, Wb)                    # not a whole number of 32-bit words
    with pytest.raises((ValueError, RuntimeError)):
        m.decompress_batch(st, Hb + 4, Wb)                         # more blocks than were coded
    with pytest.raises((ValueError, RuntimeError)):
        m.decompress_batch([b"XXXX" + st[0][4:]], Hb, Wb, fmt="rows")   # not an 'LBW1' container
    with pytest.raises(ValueError):
        m.compress_batch(x[..., :-1].contiguous())                 # wrong channel count
    with pytest.raises(ValueError):
        m.forward(x.permute(0, 3, 1, 2), x.permute(0, 3, 1, 2)[:, :, :1])
    # the handle still works afterwards
    assert torch.equal(m.decompress_batch(st, Hb, Wb), r["zhat"])


@pytest.mark.parametrize("name", ["tiny_ks3111", "tiny_ks3311"])
def test_validate_recu_reco_matches_reference(name):
    """The recursive reconstruction of validate_recu_reco_fast on the GPU against the reference's own loop:
    zhat within 1e-5 relative, self-information within 1e-4 relative; teacher-forced forward() on its result
    reproduces it bit for bit (same semantics by construction); for KS3111 it equals compress()."""
    g = load_golden("recu_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    x = torch.from_numpy(g["x"]).permute(2, 0, 1)[None].cuda()
    zhat, info = m.validate_recu_reco(x)
    z = zhat[0].permute(1, 2, 0).cpu().numpy()
    inf = info[0].permute(1, 2, 0).cpu().numpy()
    assert_rel(z, g["zhat"], what="zhat")
    assert (np.abs(inf - g["self_info"]) <= 1e-4 * np.maximum(1.0, np.abs(g["self_info"]))).all()
    xhat, info_f = m.forward(zhat, x)
    assert torch.equal(torch.clamp(xhat, -0.5, 0.5), zhat) and torch.equal(info_f, info)
    if arch.KS[1] == 1:
        r = m.compress_batch(x.permute(0, 2, 3, 1).contiguous(), want_bits=True)
        assert torch.equal(r["zhat"].permute(0, 3, 1, 2), zhat)


@pytest.mark.parametrize("name,n_img", [("tiny_ks3111", 83), ("tiny_ks3311", 150), ("b8_lowrate_2rows", 96)])
def test_gang_decode_many_rows(name, n_img):
    """Decoder raster steps with n_img > 64 rows (several batches decoded in one raster pass, as bench.py's
    pipeline does) stay on the latency-shaped kernel (LBIC_DEC_SMALL_MAX, default 1024) and must reproduce the
    encoder's reconstruction bit-exactly, also for row counts that are not a multiple of the 16-row tile."""
    g = load_golden("loop_" + name)
    arch = golden_arch(g)
    m = model_for(arch, int(g["weight_seed"]))
    x0 = torch.from_numpy(g["x"])[None].cuda()
    noise = torch.rand((n_img - 1,) + tuple(x0.shape[1:]), generator=torch.Generator().manual_seed(7)).cuda() - 0.5
    x = torch.cat([x0, noise])
    r = m.compress_batch(x)
    assert np.array_equal(r["symbols"][0].cpu().numpy(), g["symbols"])
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    zdec = m.decompress_batch(streams, *g["x"].shape[:2])
    assert torch.equal(zdec, r["zhat"]), "ganged decode differs from the encoder's reconstruction"
    # and as two passes of the same handle with different row counts (graphs rebuilt per shape)
    z2 = m.decompress_batch(streams[:17], *g["x"].shape[:2])
    assert torch.equal(z2, r["zhat"][:17])


@pytest.mark.parametrize("shape", [(8, 12), (5, 1), (1, 7), (6, 2)])
def test_layer0_cache_equals_five_positions(shape, monkeypatch):
    """KS[1] = 3: the context net's layer-0 map cache (codec.hip, computed once per block at its own step, border
    columns at the steps that own them) gives bit-identical symbols, indexes, bits and reconstructions to layer 0
    evaluated at the five positions of every block (LBIC_L0CACHE=0), for compress(), the raster and the wavefront
    (sub-stream) decoders and the validation loop's frame padding; ragged and one-block-wide frames included."""
    from lbic.model import BlockBasedImgCompLossyNetv9
    g = load_golden("loop_tiny_ks3311")
    arch = golden_arch(g)
    sd = synth_state_dict(arch, int(g["weight_seed"]))
    cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
    models = {}
    for on in ("0", "1"):
        monkeypatch.setenv("LBIC_L0CACHE", on)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(sd)
        m.update(force=True)
        models[on] = m
    Hb, Wb = shape
    rng = np.random.default_rng(11)
    xb = torch.from_numpy(np.stack([rng.random((Hb, Wb, arch.cx), dtype=np.float32) - 0.5 for _ in range(3)])).cuda()
    r = {k: m.compress_batch(xb, want_bits=True) for k, m in models.items()}
    for key in ("symbols", "indexes", "bits", "zhat"):
        assert torch.equal(r["0"][key], r["1"][key]), key
    m1 = models["1"]
    st = m1.entropy_encode(r["1"]["symbols"], r["1"]["indexes"])
    assert torch.equal(m1.decompress_batch(st, Hb, Wb), r["1"]["zhat"])
    rows = m1.entropy_encode(r["1"]["symbols"], r["1"]["indexes"], fmt="rows", Hb=Hb, Wb=Wb)
    assert torch.equal(m1.decompress_batch(rows, Hb, Wb, fmt="rows"), r["1"]["zhat"])
    v = {k: m.validate_recu_reco(xb.permute(0, 3, 1, 2)) for k, m in models.items()}
    assert torch.equal(v["0"][0], v["1"][0]) and torch.equal(v["0"][1], v["1"][1])


def test_sibling_handles_share_weights():
    """lbc_create_sibling: a second handle on the same packed weights codes bit-identically (its own workspace,
    graphs and tables), decodes the first handle's streams, and keeps its weights when the source handle is
    re-finalized with another state dict."""
    from lbic.model import BlockBasedImgCompLossyNetv9
    g = load_golden("loop_tiny_ks3311")
    arch = golden_arch(g)
    cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, int(g["weight_seed"])))
    m.update(force=True)
    sib = m.sibling()
    x = torch.from_numpy(g["x"])[None].cuda()
    r, rs = m.compress_batch(x), sib.compress_batch(x)
    for key in ("symbols", "indexes", "zhat"):
        assert torch.equal(r[key], rs[key]), key
    assert np.array_equal(rs["symbols"][0].cpu().numpy(), g["symbols"])
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    assert torch.equal(sib.decompress_batch(streams, *g["x"].shape[:2]), r["zhat"])
    m.load_state_dict(synth_state_dict(arch, int(g["weight_seed"]) + 1))      # source re-finalized
    assert not torch.equal(m.compress_batch(x)["symbols"], r["symbols"])
    assert torch.equal(sib.compress_batch(x)["symbols"], r["symbols"])
    del m
    assert torch.equal(sib.decompress_batch(streams, *g["x"].shape[:2]), r["zhat"])


def test_failed_finalize_keeps_the_working_weights():
    """lbc_finalize packs into a new weight set and installs it only when every layer packed: on a sibling
    (no host tensors) it fails and the sibling keeps coding with its shared weights; a re-finalize of the source with a
    new state dict rebuilds the team program (keyed on the packed set's id, not on reusable addresses)."""
    import ctypes
    from lbic import _lib
    from lbic.model import BlockBasedImgCompLossyNetv9, decompress_teams
    g = load_golden("loop_tiny_ks3311")
    arch = golden_arch(g)
    cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
    m = BlockBasedImgCompLossyNetv9(cfg)
    m.load_state_dict(synth_state_dict(arch, int(g["weight_seed"])))
    m.update(force=True)
    sib = m.sibling()
    x = torch.from_numpy(g["x"])[None].cuda()
    r = m.compress_batch(x)
    assert _lib.lib().lbc_finalize(sib._h) != 0              # a sibling holds no host tensors: packing fails ...
    rs = sib.compress_batch(x)                                # ... and it still codes with the shared weights
    assert torch.equal(rs["symbols"], r["symbols"]) and torch.equal(rs["zhat"], r["zhat"])
    streams = m.entropy_encode(r["symbols"], r["indexes"])
    Hb, Wb = g["x"].shape[:2]
    z1 = decompress_teams([m, sib], [streams, streams], Hb, Wb)
    assert torch.equal(z1[0], r["zhat"]) and torch.equal(z1[1], r["zhat"])
    # re-finalize the source with other weights: the recorded team program must follow the new weight set
    m.load_state_dict(synth_state_dict(arch, int(g["weight_seed"]) + 3))
    m.update(force=True)
    r2 = m.compress_batch(x)
    s2 = m.entropy_encode(r2["symbols"], r2["indexes"])
    sib2 = m.sibling()
    z2 = decompress_teams([m, sib2], [s2, s2], Hb, Wb)
    assert torch.equal(z2[0], r2["zhat"]) and torch.equal(z2[1], r2["zhat"])
