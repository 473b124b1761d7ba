"""GPU rANS decoder (k_rans_decode through lbc_rans_decode_gpu, the kernel lbc_decode runs once per raster
step) against the oracle coder (oracle/rans_oracle.c, a restatement of CompressAI's RansDecoder):
decode(encode) bit-exact for every table, for symbols far outside the tables (bypass escapes with up to 8
4-bit chunks), for latent widths that are not a multiple of the 64-lane chunk, for ragged stream counts,
and loud errors on truncated streams.  Parity with CompressAI's own bytes is unpinned."""
import numpy as np
import pytest
import torch

from lbic.arch import Arch
from oracle import oracle as O
from test_gpu_parity import model_for

pytestmark = pytest.mark.gpu


@pytest.fixture(autouse=True, params=["lds", "sparse"])
def rans_variant(request, monkeypatch):
    """Both decoder variants: the LDS table image (k_rans_decode) and the sparse one (centre-interval fast path,
    tables read from global memory, k_rans_decode_sparse); lbc_decode picks by bits per symbol."""
    monkeypatch.setenv("LBIC_RANS_SPARSE", "1" if request.param == "sparse" else "0")
    return request.param


def _symbols(rng, tabs, idx, wide):
    """Gaussian draws at 1.3x the table scale (mostly inside the table), plus `wide` extreme values."""
    scale = np.asarray(tabs.table, np.float64)[idx]
    s = np.rint(rng.normal(0.0, 1.3, idx.shape) * scale).astype(np.int64)
    flat = s.reshape(-1)
    pos = rng.choice(flat.size, size=min(wide, flat.size), replace=False)
    flat[pos] = rng.choice([-(2 ** 26), -70000, -5000, 5000, 70000, 2 ** 26], size=pos.size)   # raw < 2^28 (8 chunks)
    return s.astype(np.int32)


@pytest.mark.parametrize("M,n,chunks", [(16, 7, 9), (96, 32, 4), (208, 5, 3), (256, 3, 2)])
def test_gpu_decode_roundtrip(M, n, chunks):
    m = model_for(Arch(8, (3, 1, 1, 1), 64, M))
    tabs = O.GaussianTables()
    rng = np.random.default_rng(M * 1000 + n)
    idx = rng.integers(0, 64, (chunks, n, M)).astype(np.int32)
    idx[0, 0, :] = np.arange(M) % 64                      # every table at least once
    sym = _symbols(rng, tabs, idx, wide=3 * n)
    streams = [tabs.encode(sym[:, k].reshape(-1), idx[:, k].reshape(-1)) for k in range(n)]
    # the product coder writes the same bytes
    assert streams == m.entropy_encode(torch.from_numpy(sym.transpose(1, 0, 2).reshape(n, -1).copy()),
                                       torch.from_numpy(idx.transpose(1, 0, 2).reshape(n, -1).copy()))
    out = m.rans_decode_gpu(streams, torch.from_numpy(idx)).cpu().numpy()
    assert np.array_equal(out, sym)


def test_gpu_decode_short_tables_and_escapes_only():
    """Only the narrowest tables (0 and 1: a handful of symbols, the centre symbol holding almost all of
    the mass) and only escape symbols: every symbol goes through the bypass path."""
    M, n = 96, 4
    m = model_for(Arch(8, (3, 1, 1, 1), 64, M))
    tabs = O.GaussianTables()
    rng = np.random.default_rng(7)
    idx = rng.integers(0, 2, (3, n, M)).astype(np.int32)
    sym = rng.integers(-(2 ** 26), 2 ** 26, (3, n, M)).astype(np.int64)
    sym[sym % 3 == 0] = rng.integers(-40, 40)
    sym = sym.astype(np.int32)
    streams = [tabs.encode(sym[:, k].reshape(-1), idx[:, k].reshape(-1)) for k in range(n)]
    out = m.rans_decode_gpu(streams, torch.from_numpy(idx)).cpu().numpy()
    assert np.array_equal(out, sym)


def test_gpu_decode_truncated_stream_raises():
    M, n = 96, 2
    m = model_for(Arch(8, (3, 1, 1, 1), 64, M))
    tabs = O.GaussianTables()
    rng = np.random.default_rng(3)
    idx = rng.integers(40, 64, (4, n, M)).astype(np.int32)
    sym = _symbols(rng, tabs, idx, wide=0)
    streams = [tabs.encode(sym[:, k].reshape(-1), idx[:, k].reshape(-1)) for k in range(n)]
    with pytest.raises(RuntimeError):
        m.rans_decode_gpu([streams[0], streams[1][:16]], torch.from_numpy(idx))
    with pytest.raises(ValueError):
        m.rans_decode_gpu(streams, torch.from_numpy(idx[:, :1]))
    # the handle still decodes afterwards
    assert np.array_equal(m.rans_decode_gpu(streams, torch.from_numpy(idx)).cpu().numpy(), sym)


def test_gpu_decode_low_rate_mostly_centre():
    """The regime of the B8_lowrate operating point: almost every symbol is the table's centre (value 0), a few
    +-1 / +-2 and rare escapes, over every table."""
    M, n = 96, 32
    m = model_for(Arch(8, (3, 1, 1, 1), 64, M))
    tabs = O.GaussianTables()
    rng = np.random.default_rng(11)
    idx = rng.integers(0, 64, (6, n, M)).astype(np.int32)
    sym = np.zeros(idx.shape, np.int32)
    flat = sym.reshape(-1)
    pos = rng.choice(flat.size, size=flat.size // 50, replace=False)
    flat[pos] = rng.choice([-2, -1, 1, 2, 3000], size=pos.size)
    streams = [tabs.encode(sym[:, k].reshape(-1), idx[:, k].reshape(-1)) for k in range(n)]
    out = m.rans_decode_gpu(streams, torch.from_numpy(idx)).cpu().numpy()
    assert np.array_equal(out, sym)
