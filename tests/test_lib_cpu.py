"""CPU-side checks of liblbic.so (no GPU needed): the library loads, exports every symbol include/lbic.h
declares, and its host C++ entropy coder agrees with the oracle (pmf_to_quantized_cdf tables bit-exact,
rANS bitstreams byte-identical, round trips exact)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, load_golden
from lbic import _lib
from oracle import oracle as O


def test_header_symbols_exported():
    hdr = open(os.path.join(ROOT, "include", "lbic.h")).read()
    declared = set(re.findall(r"\b(lbc_[a-z_0-9]+)\s*\(", hdr))
    assert declared == set(_lib.EXPORTS)
    lib = _lib.lib()
    for name in declared:
        assert hasattr(lib, name), name


def _tables_from_golden():
    g = load_golden("cdf_pmf")
    probs = np.split(g["prob"], np.cumsum(g["prob_len"])[:-1])
    return g, probs


def test_pmf_to_quantized_cdf_matches_oracle():
    from lbic.entropy import pmf_to_quantized_cdf
    _, probs = _tables_from_golden()
    for p in probs:
        ours = pmf_to_quantized_cdf(p).numpy()
        assert np.array_equal(ours, O.pmf_to_quantized_cdf(p))


def test_gaussian_update_matches_reference_pmfs():
    """entropy.GaussianConditional.update builds the same tables as the oracle from the reference pmfs."""
    from lbic.entropy import GaussianConditional, get_scale_table
    g, probs = _tables_from_golden()
    gc = GaussianConditional()
    gc.update_scale_table(get_scale_table(), force=True)
    assert np.array_equal(gc.scale_table.numpy().view(np.uint32), g["scale_table"].view(np.uint32))
    assert np.array_equal(gc.offset.numpy(), g["offset"])
    assert np.array_equal(gc.cdf_length.numpy(), g["cdf_length"])
    ref = O.GaussianTables(probs)
    assert np.array_equal(gc.quantized_cdf.numpy()[:, :ref.cdf.shape[1]], ref.cdf)


def _host_model(tabs):
    L = _lib.lib()
    cfg = _lib.LbcConfig()
    cfg.block_size, cfg.n, cfg.m, cfg.device = 4, 64, 16, 0
    for i, k in enumerate((3, 1, 1, 1)):
        cfg.ks[i] = k
    h = ctypes.c_void_p()
    _lib.check(L.lbc_create(ctypes.byref(cfg), ctypes.byref(h)))
    _lib.check(L.lbc_set_entropy_tables(h, _lib.ptr(tabs.table), 64, _lib.ptr(tabs.cdf), tabs.cdf.shape[1],
                                        _lib.ptr(tabs.cdf_length), _lib.ptr(tabs.offset)))
    return h


def test_rans_host_matches_oracle_bytes():
    _, probs = _tables_from_golden()
    tabs = O.GaussianTables(probs)
    h = _host_model(tabs)
    L = _lib.lib()
    rng = np.random.default_rng(7)
    for n in (1, 96, 5000):
        idx = rng.integers(0, 64, n).astype(np.int32)
        sym = np.rint(rng.standard_normal(n) * tabs.table[idx] * 1.3).astype(np.int32)
        sym[::53] = rng.integers(-3000, 3000, len(sym[::53]))     # exercise the bypass escape
        p, ln = ctypes.c_void_p(), ctypes.c_size_t()
        _lib.check(L.lbc_rans_encode(h, _lib.ptr(sym), _lib.ptr(idx), n, ctypes.byref(p), ctypes.byref(ln)))
        ours = ctypes.string_at(p, ln.value)
        L.lbc_free(p)
        assert ours == tabs.encode(sym, idx)
        buf = np.frombuffer(ours, np.uint8).copy()
        out = np.zeros(n, np.int32)
        _lib.check(L.lbc_rans_decode_host(h, _lib.ptr(buf), len(buf), _lib.ptr(idx), n, _lib.ptr(out)))
        assert np.array_equal(out, sym)
    L.lbc_destroy(h)


def test_golden_symbols_encode_identically():
    """The reference closed loop's own (symbols, indexes) encode to the same bytes in both coders."""
    _, probs = _tables_from_golden()
    tabs = O.GaussianTables(probs)
    h = _host_model(tabs)
    L = _lib.lib()
    g = load_golden("loop_b8_lowrate_2rows")
    s, i = g["symbols"].astype(np.int32), g["indexes"].astype(np.int32)
    p, ln = ctypes.c_void_p(), ctypes.c_size_t()
    _lib.check(L.lbc_rans_encode(h, _lib.ptr(s), _lib.ptr(i), len(s), ctypes.byref(p), ctypes.byref(ln)))
    assert ctypes.string_at(p, ln.value) == tabs.encode(s, i)
    L.lbc_free(p)
    L.lbc_destroy(h)


def test_errors_are_loud():
    L = _lib.lib()
    with pytest.raises(RuntimeError):
        _lib.check(L.lbc_create(None, None))
    bad = np.array([-1.0, 0.5], np.float32)
    out = np.zeros(3, np.uint32)
    with pytest.raises(RuntimeError):
        _lib.check(L.lbc_pmf_to_quantized_cdf(_lib.ptr(bad), 2, 16, _lib.ptr(out)))


def test_set_option_ranges():
    """lbc_set_option (host-only, no GPU): every option's range is checked, LBC_OPT_ENC_FORK takes -1 / 0 / 1 (the
    encoder graph forked by the pass's row count, one chain, forked), an unknown option is an error."""
    L = _lib.lib()
    cfg = _lib.LbcConfig()
    cfg.block_size, cfg.n, cfg.m, cfg.device = 4, 64, 16, 0
    for i, k in enumerate((3, 1, 1, 1)):
        cfg.ks[i] = k
    h = ctypes.c_void_p()
    _lib.check(L.lbc_create(ctypes.byref(cfg), ctypes.byref(h)))
    try:
        for opt, good, bad in ((1, (0, 65536), (-1, 160 * 1024 + 1)), (2, (1, 2), (0, 3)), (3, (0, 32), (-1, 33)),
                               (4, (-1, 0, 1), (-2, 2))):
            for v in good:
                assert L.lbc_set_option(h, opt, v) == 0, (opt, v)
            for v in bad:
                assert L.lbc_set_option(h, opt, v) != 0, (opt, v)
        assert L.lbc_set_option(h, 99, 0) != 0
    finally:
        L.lbc_destroy(h)
