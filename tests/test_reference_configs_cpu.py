"""The reference's own four configs (shipped verbatim in learned-block-based-image-compression_amd/configs/; only
``valid_data`` is redirected to a local PNG folder) through this repository's main.py: JSON parsing, the multi-lambda
sweep (main.py:17-27 of the reference), process_config's experiment layout (utils/config.py:69-102), agent dispatch by
name and the agent's construction up to the device check, which on this GPU-less host must be the loud "no GPU" error
(no CPU fallback).  The same flow runs end to end on the GPU in tests/test_agent_gpu.py (B8_lowrate at 768x768).

Also: bench.py's multi-GPU launcher and its per-image record gather (gloo, world size 2)."""
import glob
import json
import os

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# the reference's four configs, shipped verbatim (data) with the package
REF_CONFIGS = sorted(glob.glob(os.path.join(ROOT, "learned-block-based-image-compression_amd", "configs", "*.json")))


def test_shipped_configs_are_verbatim():
    """learned-block-based-image-compression_amd/configs/*.json are byte copies of the reference's configs/*.json
    (compared where /root/reference is present, i.e. not on the GPU box)."""
    assert len(REF_CONFIGS) == 4
    ref_dir = "/root/reference/configs"
    if not os.path.isdir(ref_dir):
        pytest.skip("reference not present")
    for p in REF_CONFIGS:
        with open(p, "rb") as a, open(os.path.join(ref_dir, os.path.basename(p)), "rb") as b:
            assert a.read() == b.read(), p


@pytest.mark.parametrize("path", REF_CONFIGS, ids=[os.path.basename(p) for p in REF_CONFIGS])
def test_reference_config_runs_through_main(path, tmp_path, monkeypatch):
    from PIL import Image
    import main as lbic_main
    from lbic.arch import arch_from_config
    from lbic.config import AttrDict
    raw = json.load(open(path))
    data = tmp_path / "valid"
    data.mkdir()
    Image.fromarray(np.zeros((16, 16, 3), np.uint8)).save(data / "a.png")
    cfg = dict(raw)
    cfg["valid_data"] = str(data)                       # the only override
    assert set(cfg) == set(raw)
    p = tmp_path / os.path.basename(path)
    p.write_text(json.dumps(cfg))
    monkeypatch.chdir(tmp_path)
    arch = arch_from_config(AttrDict(cfg))
    assert (arch.B, list(arch.KS), arch.N, arch.M) == (raw["block_size"], raw["KS"], raw["N"], raw["M"])
    seen = []
    real = lbic_main.AGENTS["BlockBasedImgCompLossyAgent"]

    class Probe(real):
        def __init__(self, config):
            seen.append((config.exp_name, config.lambda_, config.mode, config.log_dir))
            super().__init__(config)            # -> the device check (no GPU here)

    monkeypatch.setitem(lbic_main.AGENTS, "BlockBasedImgCompLossyAgent", Probe)
    with pytest.raises(RuntimeError, match="no GPU is visible"):
        lbic_main.main([str(p)])
    lam = raw["lambda_"][0] if raw.get("multi_agent") else raw["lambda_"]
    exp, got_lam, mode, log_dir = seen[0]
    assert got_lam == lam and mode == raw["mode"]
    if raw.get("multi_agent"):
        assert exp == os.path.join(raw["multi_exp_name"], "exp_" + str(lam))
    # (logging is set up once per process, as the reference's run_once setup_logging, utils/config.py:24)
    assert all(os.path.isdir(os.path.join(log_dir, "..", d)) for d in ("summaries", "checkpoints", "out", "logs"))


def test_bench_relaunch_command(monkeypatch):
    """--gpus N without WORLD_SIZE re-runs bench.py under torch.distributed.run (one process per GPU, 127.0.0.1)
    as a child process and exits with its code."""
    import sys
    import bench
    calls = []
    monkeypatch.setattr(bench.subprocess, "call", lambda cmd: calls.append(cmd) or 7)
    monkeypatch.setattr(sys, "argv", ["bench.py", "--gpus", "4", "--steps", "3"])
    args = bench.parse_args()
    assert bench.relaunch_distributed(args) == 7
    cmd = calls[0]
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "127.0.0.1" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"]


def _gather_worker(rank, world, port, out):
    import torch
    import torch.distributed as dist
    import bench
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rec = torch.tensor([[100.0 + rank, 5.0 * rank, 12.0], [200.0 + rank, 1.0, 12.0]], dtype=torch.float64)
    allrec, ok = bench.gather_records(rec, rank != 7, True)
    if rank == 0:
        np.save(out, allrec.numpy())
        assert ok
    dist.destroy_process_group()


def test_bench_gather_records_gloo(tmp_path):
    import socket
    import torch.multiprocessing as mp
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = str(tmp_path / "rec.npy")
    mp.spawn(_gather_worker, args=(2, port, out), nprocs=2, join=True)
    rec = np.load(out)
    assert rec.shape == (4, 3)
    assert list(rec[:, 0]) == [100.0, 200.0, 101.0, 201.0]


def test_bench_roofline_dominance_is_wall_occupancy():
    """bench.py's roofline picks the dominant kernel by wall occupancy in the timed region: the team
    decoder's summed launch durations against the encoder graphs' wall time -- not the encoder launches' summed
    durations, which exceed the graphs' wall time because the forked branches overlap."""
    import bench
    dt, steps = 4.5, 20
    # encoder: 100,000 launches of 50 us each (5.0 s summed) inside 3.5 s of graph wall time; team: 3 launches, 3.9 s
    kstats = {"k_gemm_t": dict(launches=1000, total_launches=100000, total_ms=50.0, flops=1e12, bytes=9e9,
                               total_flops=1e17, total_bytes=9e14),
              "k_gemm_s": dict(launches=10, total_launches=500, total_ms=0.05, flops=1e9, bytes=1e8,
                               total_flops=5e11, total_bytes=5e10)}
    enc = dict(ms=3500.0, passes=20)
    team = dict(launches=3, ms=3900.0, bytes=3 * 1.9e12, flops=3 * 2.8e13, steps=20 * 9216, plain=[1, 1, 1],
                timeouts=0, hw=9216, windows=[[0.4, 1.7, 4, 4], [1.8, 3.1, 8, 8], [3.2, 4.5, 8, 8]], enc_done=3.1)
    roof, kernels = bench.roofline(kstats, dt, team, enc, steps)
    assert roof["kernel"] == "k_dec_team", roof
    assert roof["wall_occupancy_ms_per_step"] <= dt / steps * 1e3      # the dominant kernel fits in the step
    assert kernels["k_gemm_t"]["summed_launch_s"] > kernels["k_gemm_t"]["wall_occupancy_s"]
    agg = roof["per_kernel"]["k_gemm_t"]["aggregate"]
    assert abs(agg["achieved_tflops"] - (1e17 + 5e11) / 3.5 / 1e12) < 1e-2
    assert abs(roof["achieved"] - 1.9e12 / 1.3 / 1e9) < 1.0 and roof["bound"] == "hbm"
    # a faster decoder: the encoder graphs become the dominant family
    team["ms"] = 2000.0
    roof, _ = bench.roofline(kstats, dt, team, enc, steps)
    assert roof["kernel"] == "k_gemm_t" and roof["bound"] == "mfma"


def test_bench_roofline_single_chain_encoder():
    """Multi-batch encoder passes run the encoder graph as ONE chain of launches (LBC_OPT_ENC_FORK 0): the k_gemm launch
    duration of the bench line is then the graphs' HIP-event wall time over their launches (an upper bound incl. the
    dependent-launch gap), the in-kernel stamps reported beside it; the per-launch work is the family's total over its
    launches."""
    import bench
    dt, steps = 4.6, 32
    kstats = {"k_gemm": dict(launches=2600, total_launches=41184, total_ms=2600 * 0.0866, flops=4.3e9, bytes=3.6e7,
                             total_flops=41184 * 4.12e9, total_bytes=41184 * 3.5e7)}
    enc = dict(ms=41184 * 0.0781, passes=8, chain=True)
    team = dict(launches=2, ms=2800.0, bytes=2 * 1.9e12, flops=2 * 2.8e13, steps=32 * 9216, plain=[1, 1],
                timeouts=0, hw=9216, windows=[[1.1, 2.8, 16, 16], [3.3, 4.5, 16, 16]], enc_done=3.3)
    roof, kernels = bench.roofline(kstats, dt, team, enc, steps)
    k = kernels["k_gemm"]
    assert roof["kernel"] == "k_gemm" and roof["bound"] == "mfma"
    assert abs(k["avg_launch_us"] - 78.1) < 0.01 and abs(k["stamped_span_us"] - 86.6) < 0.01
    assert abs(roof["achieved"] - 4.12e9 / 78.1e-6 / 1e12) < 1e-3
    enc["chain"] = False          # a forked graph: the stamps give the launch's own duration
    _, kernels = bench.roofline(kstats, dt, team, enc, steps)
    assert abs(kernels["k_gemm"]["avg_launch_us"] - 86.6) < 0.01


def test_bench_team_schedule_defaults():
    """The headline's team schedule (bench.py defaults): 16 teams per launch, ONE 32-frame batch per team (each decode
    pass decodes exactly one batch of the config), the first launch's footprint chosen by its team count (-1: 12
    workgroups per XCD slot up to 8 teams, every CU beyond), four batches per encoder wavefront pass, the encoder's
    copies on a stream of their own; two batches per team only for batches of at most 16 frames (configs 3 and 5)."""
    import bench
    a = bench.parse_args([])
    assert (a.team, a.team_batches, a.first_team_size, a.batch) == (16, 1, -1, 32)
    assert (a.enc_pass, a.d2h_stream, a.steps) == (4, 1, 32)
    assert bench.parse_args(["--batch", "8"]).team_batches == 2
    assert bench.parse_args(["--batch", "24"]).team_batches == 1
    assert bench.parse_args(["--team-batches", "2"]).team_batches == 2
