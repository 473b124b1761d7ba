"""CPU tests of the host mirror: config handling, layout, metrics, and the multi-process image sharding +
summary all-gather (gloo, world_size 2) that the GPU path uses over RCCL."""
import json
import os

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, load_golden


def test_config_and_process(tmp_path):
    from lbic.config import get_config_from_json, process_config
    cfg_path = os.path.join(PKG, "configs", "blkbsdimgcomp_B8_lowrate.json")
    cfg, d = get_config_from_json(cfg_path)
    assert cfg.block_size == 8 and cfg.N == 768 and cfg.M == 96 and cfg.agent == "BlockBasedImgCompLossyAgent"
    cfg.exp_name = os.path.join(cfg.multi_exp_name, "exp_117.045")
    cfg = process_config(cfg, root=str(tmp_path))
    assert os.path.isdir(cfg.checkpoint_dir) and os.path.isdir(cfg.log_dir)
    from lbic.arch import arch_from_config
    a = arch_from_config(cfg)
    assert a.lru == 1 and a.live_macs_per_block() == (8994816, 5925888)


def test_torch_layout_matches_reference_golden():
    from lbic.layout import arrange_block_pixels_to_channel_dim, arrange_channel_dim_to_block_pixels
    g = load_golden("loop_b4_highrate")
    img = torch.from_numpy(g["image"].astype(np.float32) / 255.0 - 0.5)[None]
    t = arrange_block_pixels_to_channel_dim(img, 4)
    assert np.array_equal(t[0].permute(1, 2, 0).numpy(), g["x"])
    assert torch.equal(arrange_channel_dim_to_block_pixels(t, 4), img)


def test_ms_ssim_sanity():
    from lbic.metrics import ms_ssim
    g = torch.Generator().manual_seed(0)
    x = torch.rand(1, 3, 192, 192, generator=g)
    assert abs(ms_ssim(x, x).item() - 1.0) < 1e-6
    a = ms_ssim(x, (x + 0.05 * torch.randn(x.shape, generator=g)).clamp(0, 1)).item()
    b = ms_ssim(x, (x + 0.20 * torch.randn(x.shape, generator=g)).clamp(0, 1)).item()
    assert 1.0 > a > b > 0.0


def _worker(rank, world, port, q):
    import torch.distributed as dist
    from lbic import dist as D
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    items = list(range(7))
    mine = D.shard(items, rank, world)
    rec = torch.tensor([[i, i * 10.0] for i in mine], dtype=torch.float64)
    allrec = D.gather_records(rec)
    q.put((rank, mine, allrec.numpy().tolist()))
    dist.destroy_process_group()


def test_shard_and_gather_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 29500 + os.getpid() % 1000
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res.sort()
    assert res[0][1] == [0, 2, 4, 6] and res[1][1] == [1, 3, 5]
    for _, _, allrec in res:
        got = sorted(int(r[0]) for r in allrec)
        assert got == list(range(7))
        assert all(r[1] == r[0] * 10 for r in allrec)


def test_band_rows_cover_the_frame():
    from lbic.band import band_rows, wavefront_steps
    for Hb in (1, 5, 6, 96, 128):
        for P in range(1, min(Hb, 8) + 1):
            b = band_rows(Hb, P)
            assert [v for v, _ in b] == list(np.cumsum([0] + [r for _, r in b])[:-1])
            assert sum(r for _, r in b) == Hb and max(r for _, r in b) - min(r for _, r in b) <= 1
    assert wavefront_steps(96, 96) == 286
    with pytest.raises(ValueError):
        band_rows(3, 4)


def test_transform_weights_are_a_codec():
    """lbic.weights.transform_state_dict: the block DCT is orthonormal in lbic.layout's channel order, and the CPU
    oracle's closed loop (compress -> rANS bytes) on a structured synthetic frame reconstructs it at a real operating
    point (tens of dB at well under 1 bpp)."""
    from lbic.arch import Arch
    from lbic.layout import image_to_blocks
    from lbic.weights import _block_dct, smooth_frame, transform_state_dict
    from oracle import oracle as O
    T = _block_dct(8)
    assert np.abs(T @ T.T - np.eye(192)).max() < 1e-12
    arch = Arch(8, (3, 1, 1, 1), 768, 96)
    sd = transform_state_dict(arch)
    xb = image_to_blocks(smooth_frame(3, 64, 64).astype(np.float32) / 255 - 0.5, 8)
    r = O.OracleCodec(arch, sd).compress(xb)
    psnr = -10 * np.log10(np.mean((r["zhat"] - xb) ** 2))
    bpp = len(r["bytes"]) * 8 / (64 * 64)
    assert psnr > 28 and bpp < 1.5, (psnr, bpp)
    with pytest.raises(ValueError):
        transform_state_dict(Arch(4, (3, 3, 1, 1), 512, 96))    # 96 coefficients > 3 * 4^2


def test_bench_team_group_sizes():
    """bench.py's team schedule never asks for more teams than one launch holds: odd batch counts at two
    batches per team and one batch per team on a full group are split; explicit --team-sizes are validated."""
    import bench
    f = bench.team_group_sizes
    assert f(20, 16, 1) == [4, 16]                       # the driver's command: partial group first
    assert f(32, 16, 1) == [16, 16]
    assert f(17, 16, 2) == [1, 16]                       # 17 at two per team would be 17 one-batch teams
    assert f(33, 16, 2) == [1, 32]
    assert f(32, 16, 2, first_tb=1) == [16, 16]          # --first-team-batches 1 on a full group of 32
    assert f(10, 16, 2, order="first-full") == [10]
    for steps in range(1, 70):
        for tb in (1, 2):
            for first in (0, 1, 2):
                sizes = f(steps, 16, tb, first_tb=first)
                assert sum(sizes) == steps
                for i, s in enumerate(sizes):
                    t = first if i == 0 and first else tb
                    assert 1 <= (s // t if s % t == 0 else s) <= 16
    with pytest.raises(SystemExit):
        f(20, 16, 1, explicit="3,17")                    # 17 one-batch teams
    with pytest.raises(SystemExit):
        f(20, 16, 1, explicit="4,15")                    # does not sum to 20
    assert f(20, 16, 1, explicit="4,16") == [4, 16]
    assert bench.first_wg_per_xcd(4, 12) == 12 and bench.first_wg_per_xcd(16, 12) == 24
