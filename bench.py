#!/usr/bin/env python3
"""Benchmark: Mpixels/s encode+decode of the block-level masked-conv codec (BASELINE.json metric).

Workload (BASELINE.json configs[1]): B8_lowrate (B=8, KS=3,1,1,1, N=768, M=96), batches of 32 synthetic
768x768 frames per GPU, in the reference bitstream format (one raster rANS stream per image).  One step =
the reference's timed region of eval_model (agents/blkbsdimgcomp_agent.py:591-599) for one 32-frame batch:
compress (GPU wavefront closed loop + host rANS encode) and decompress (GPU raster closed loop with GPU
rANS decode).  Four batches share one 128-frame encoder wavefront pass (`--enc-pass`; every launch of the encoder's
GEMMs has four times the rows, its partly filled last round of workgroups amortised over more frames), and every batch
is entropy coded and decoded as its own 32-frame raster pass (one team of workgroups per batch); the line reports the
one-batch-per-pass schedule beside it (`one_batch_per_encode_pass`).

Schedule of the headline (`value`, `--team 16`, the default): one encoder handle compresses batch after batch on its
own HIP stream (host rANS on helper threads); every 16 encoded batches (the first group: the remainder) are decoded
by ONE persistent k_dec_team launch (lbc_decode_team: one team of workgroups per 32-frame batch, two teams per XCD,
team barriers instead of kernel boundaries) on a second stream, beside the encoder's next batches; the first launch
takes part of every XCD's CUs with up to 8 teams (`--first-team-size`: 12 of 32), every CU with 9-16 (the driver's 32
batches: two launches of 16).  `--team 0` selects the
`--workers` schedule (W codec handles on the shared weights, each compressing, entropy coding and decoding whole
batches) or, with `--workers 0`, the encoder + `--depth` decoders pipeline.  The timed region holds exactly the `--steps` compressions and the `--steps`
decompressions of the same batches, fill and drain included; inputs are resident in HBM when it starts.  Reported
beside it: the same schedule with 8 whole-XCD teams per launch (`eight_teams_per_launch`), one decode pass in flight
(`one_decode_in_flight`), no overlap at all (`serial_schedule`), the gang
schedule (`gang_schedule`: one raster pass over several queued batches, more frames in flight, not the headline),
and the opt-in sub-stream format (`substream_format`, not the reference bitstream).

Weights: the seeded synthetic set (lbic.weights) at the config's operating point (`--rate low`: about
0.13 bpp on these frames, BASELINE.md's B8_lowrate point is 0.117 bpp); `--rate high` is the 12 bpp set.
Frames: seeded uint8 noise (no Kodak, no checkpoints offline).

Multi-GPU: `--gpus N` relaunches itself under torch.distributed.run (one process per GPU, 127.0.0.1)
unless WORLD_SIZE is already set.  Images are sharded (every rank codes its own batches: weak scaling);
the only collectives are barriers, a MAX of the timed region and one all_gather of the per-image
rate/distortion records (RCCL over xGMI).

Prints ONE JSON line on rank 0.  Roofline, CPU baseline and PMC definitions: DESIGN.md §6.
"""
import argparse
import json
import math
import os
import platform
import queue
import re
import subprocess
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "learned-block-based-image-compression_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

METRIC = "Mpixels/s encode+decode, B8_lowrate N768M96, 768×768; bpp/PSNR vs ref"
PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 MFMA (dense) peak
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E peak (spec)

CONFIG_LAMBDA = {"B8_lowrate": 117.045, "B8_highrate": 11704.5, "B4_highrate": 11704.5, "B16_lowrate": 117.045}
CONFIGS = {   # name -> (B, KS, N, M)
    "B8_lowrate": (8, (3, 1, 1, 1), 768, 96),
    "B8_highrate": (8, (3, 3, 1, 1), 1152, 128),
    "B4_highrate": (4, (3, 3, 1, 1), 512, 96),
    "B16_lowrate": (16, (3, 1, 1, 1), 1280, 192),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=32,
                    help="timed batches (each encoded and decoded in the region; the pipeline's fill and drain -- the "
                         "first group's encodes and the last group's decode launch -- are inside it)")
    ap.add_argument("--warmup", type=int, default=8, help="untimed pipeline batches before the timed region")
    ap.add_argument("--batch", type=int, default=32, help="frames per batch (per GPU)")
    ap.add_argument("--size", type=int, default=768, help="frame width (and height unless --height)")
    ap.add_argument("--height", type=int, default=0, help="frame height (default: --size)")
    ap.add_argument("--config", default="B8_lowrate", choices=sorted(CONFIGS))
    ap.add_argument("--rate", default="", choices=("", "low", "mid", "high"),
                    help="synthetic weight operating point (default: the config's, lbic.weights.rate_for_lambda: 'low' "
                         "for the lambda-117 configs, 'mid' = ~1.6 bpp for the high-rate ones; 'high' = the 12-47 bpp set)")
    ap.add_argument("--depth", type=int, default=3, help="decode passes in flight beside the encoder (0 = serial)")
    ap.add_argument("--share-weights", type=int, default=1,
                    help="1: decoder handles share the encoder handle's device weights (lbc_create_sibling)")
    ap.add_argument("--team", type=int, default=16,
                    help="headline schedule: one encoder handle compresses the batches while groups of TEAM encoded "
                         "batches are decoded by ONE persistent team launch each (lbc_decode_team: one team of "
                         "workgroups per 32-frame batch; more than 8: two teams per XCD); 0 = the --workers / --depth "
                         "schedules")
    ap.add_argument("--team-batches", type=int, default=0, choices=(0, 1, 2),
                    help="team schedule: encoded batches per decode team (2: each team of a launch decodes the images "
                         "of two batches side by side, twice the row tiles per weight fetch; a launch then holds up to "
                         "2 x TEAM batches; 0 = auto: 2 for batches of at most 16 frames, else 1 -- the headline's "
                         "32-frame batches are decoded one per team)")
    ap.add_argument("--first-team-size", type=int, default=-1,
                    help="team schedule: workgroups per XCD slot of each team in the FIRST decode launch, the one beside "
                         "the encoder's next batches (LBC_OPT_TEAM_SIZE; 0: all).  With up to 8 teams in that launch this "
                         "is the workgroups (CUs) per XCD, the rest left to the encoder; with 9-16 teams two teams share "
                         "an XCD slot and each takes min(16, this).  -1 (default): 12 with up to 8 teams (the driver's "
                         "20 batches in round 5: 4 teams), every CU with 9-16 (32 batches: 16 teams, 120-123 vs 119-120 "
                         "Mpix/s at 12, profiles/r06/fts_*)")
    ap.add_argument("--first-team-batches", type=int, default=0, choices=(0, 1, 2),
                    help="team schedule: batches per team in the FIRST decode launch (0: --team-batches)")
    ap.add_argument("--team-sizes", default="",
                    help="team schedule: explicit batches per decode launch, comma-separated, summing to --steps "
                         "(default: from --team-groups)")
    ap.add_argument("--team-groups", default="last-full", choices=("last-full", "first-full"),
                    help="when --steps is not a multiple of --team: the partial group is the first launch (last-full) "
                         "or the last one (first-full)")
    ap.add_argument("--drain-wg-per-cu", type=int, default=1, choices=(1, 2),
                    help="team schedule: workgroups per CU of the last decode launch, which runs after the last encode "
                         "with the GPU otherwise idle (LBC_OPT_TEAM_WG_PER_CU)")
    ap.add_argument("--workers", type=int, default=4,
                    help="headline schedule: W workers, each (own handle + stream + thread) compressing, entropy coding "
                         "and decoding whole batches (0 = the encoder + --depth decoders pipeline)")
    ap.add_argument("--enc-lds-floor", type=int, default=0,
                    help="LDS bytes reserved per encoder GEMM workgroup (caps the encoder's workgroups per CU, leaving "
                         "wave slots to the decode passes; lbc_set_option LBC_OPT_ENC_LDS_FLOOR)")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (set before HIP starts, unless already in the environment): "
                         "every busy stream needs a hardware queue of its own (lbic/streams.py)")
    ap.add_argument("--sample-every", type=int, default=16, help="kernel timing-stamp sampling period (steps)")
    ap.add_argument("--enc-sample-every", type=int, default=16,
                    help="team schedule: in-kernel timing stamps in every n-th wavefront step of the encoder graph (the "
                         "k_gemm launch duration of the bench line; 0 = none: graph wall time / launches only)")
    ap.add_argument("--cpu-budget", type=float, default=24.0, help="seconds of CPU-baseline work (0 = skip)")
    ap.add_argument("--side-steps", type=int, default=2,
                    help="batches of the one-decode-in-flight and serial schedules reported beside (0 = skip)")
    ap.add_argument("--gang", type=int, default=0,
                    help="batches per raster pass of an extra gang-schedule leg (0 = skip; not in the default run, so "
                         "the same-command rocprof summary holds only the headline's kernel shapes)")
    ap.add_argument("--substream-steps", type=int, default=0, help="batches in the opt-in sub-stream format (0 = skip)")
    ap.add_argument("--encode-only", type=int, default=0, help="profiling aid: this many encoder passes, no JSON")
    ap.add_argument("--enc-pass", type=int, default=4, choices=(1, 2, 4),
                    help="team schedule: batches per encoder pass (2, 4: that many 32-frame batches in one wavefront "
                         "pass -- each launch of the encoder's GEMMs then has 2 / 4 times the rows, so its last, partly "
                         "filled round of workgroups is amortised over more frames -- each batch still entropy coded and "
                         "decoded as its own 32-frame batch; the driver's 32 batches, profiles/r06/exp/encpass_*: 1 / 2 / "
                         "4 batches per pass 119.7-120.0 / 128.0-128.4 / 130.6-130.7 Mpix/s; the line reports the one-"
                         "batch figure beside it, one_batch_per_encode_pass)")
    ap.add_argument("--d2h-stream", type=int, default=1,
                    help="team schedule, 1: the encoder's symbols / indexes go device -> host on a copy stream of their "
                         "own (ordered after the compress by an event; the entropy coder waits for the copy), so the "
                         "encoder stream starts the next batch at once; 0: on the encoder stream, synchronized")
    ap.add_argument("--per-image", type=int, default=1,
                    help="1: also time the reference's per-image path (eval_model, agents/blkbsdimgcomp_agent.py:591-599: "
                         "compress() then decompress() of ONE frame, batch 1), median of 3")
    a = ap.parse_args(argv)
    if a.team_batches == 0:
        a.team_batches = 2 if a.batch <= 16 else 1
    return a


def team_group_sizes(steps, team, tb, order="last-full", explicit="", first_tb=0, ndec=16):
    """Batches per decode launch of the team schedule.  Launch g decodes its batches as teams of tb_g batches (tb_g =
    first_tb for the first launch when given, else tb), or one batch per team when its count is not a multiple of
    tb_g; every launch may hold at most min(team, ndec, TEAM_MAX = 16) teams (one decoder handle per team).  The default
    groups are team * tb batches with the partial group first (order "last-full") or last; a group that would exceed
    the team limit (an odd count at tb = 2 past `team`, or first_tb = 1 on a full group) is split so that no launch
    does.  Explicit sizes (--team-sizes) are validated, never changed."""
    limit = min(team, ndec, 16)

    def teams_of(s, t):
        return s // t if s % t == 0 else s

    def tb_of(i):
        return first_tb if i == 0 and first_tb else tb
    if explicit:
        sizes = [int(v) for v in explicit.split(",")]
        if sum(sizes) != steps or min(sizes) < 1:
            raise SystemExit(f"--team-sizes {explicit}: must sum to {steps}, each >= 1")
        for i, s in enumerate(sizes):
            if teams_of(s, tb_of(i)) > limit:
                raise SystemExit(f"--team-sizes {explicit}: group {i} ({s} batches at {tb_of(i)} per team) needs "
                                 f"{teams_of(s, tb_of(i))} teams, at most {limit}")
        return sizes
    nfull, rem = divmod(steps, team * tb)
    sizes = ([rem] if rem else []) + [team * tb] * nfull
    if order == "first-full":
        sizes = sizes[::-1]
    out = []
    for s in sizes:
        t = tb_of(len(out))
        if teams_of(s, t) <= limit:
            out.append(s)
        elif s % t:                           # odd at two per team: one batch alone, then two per team
            out += [s % t, s - s % t]
        else:                                 # one per team past the limit: chunks of `limit`
            out += [min(limit, s - c) for c in range(0, s, limit)]
    for i, s in enumerate(out):
        assert 1 <= teams_of(s, tb_of(i)) <= limit, (out, i)
    return out


def first_wg_per_xcd(teams, team_size, cus_per_xcd=32):
    """Workgroups (one per CU) a team launch of `teams` teams at LBC_OPT_TEAM_SIZE `team_size` puts on each XCD it uses
    (lbc_decode_team's geometry, codec.hip: up to 4 teams span two XCD slots each, team_size per slot; 5-8 one slot
    each; 9-16 two teams per slot of min(16, team_size) workgroups each)."""
    if teams > 8:
        return 2 * min(cus_per_xcd // 2, team_size)
    return min(cus_per_xcd, team_size)


def relaunch_distributed(args):
    """--gpus N > 1 without a torch.distributed environment: run this script under torch.distributed.run
    (one process per GPU) as a child process -- nothing here has touched the GPU -- and exit with its code."""
    import socket
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    log("[bench] relaunch:", " ".join(cmd))
    return subprocess.call(cmd)


def cpu_info():
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return model, os.cpu_count()


def cpu_baseline(arch, sd, H, W, budget_s):
    """oracle/torch_ref.py (torch-CPU restatement of the reference's compress/decompress, parity-checked
    against the reference's golden vectors) on the host cores: encode+decode of the first R block rows of one
    frame (per-block cost is content-independent), at 1 thread (eval_model's setting,
    agents/blkbsdimgcomp_agent.py:565-566) and at every thread the box grants."""
    import numpy as np
    import torch
    from oracle import oracle as O
    from oracle.torch_ref import TorchRef
    img = np.random.default_rng(0).integers(0, 256, (3, H, W), dtype=np.uint8).astype(np.float32) / 255.0 - 0.5
    xb = O.image_to_blocks(img, arch.B)
    Hb, Wb = xb.shape[:2]
    ref = TorchRef(arch, sd)
    model, nproc = cpu_info()
    threads_all = int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or nproc
    prev = torch.get_num_threads()
    counts = sorted({t for t in (1, 4, 8, 16, threads_all) if t <= threads_all})
    res = {}
    for th in counts:
        torch.set_num_threads(th)

        def run(rows):
            t0 = time.perf_counter()
            out = ref.compress(xb, rows=rows)
            ref.decompress(out["bytes"], Hb, Wb, rows=rows)
            return time.perf_counter() - t0

        t1 = run(1)
        rows = int(max(1, min(Hb, math.floor(budget_s / len(counts) / max(t1, 1e-3)))))
        t = run(rows) if rows > 1 else t1
        res[th] = (rows * arch.B * W / t / 1e6, rows, t)
    torch.set_num_threads(prev)
    best = max(counts, key=lambda t: res[t][0])
    v_b, rows_b, t_b = res[best]
    return dict(value=round(v_b, 6), unit="Mpixels/s", cores=best, kind="port",
                sample=f"oracle/torch_ref.py (torch-CPU fp32 restatement of compress/decompress, C rANS) encode+decode "
                       f"of the first {rows_b} of {Hb} block rows of one {H}x{W} frame at {best} thread(s) "
                       f"({t_b:.1f} s), the fastest of {counts} threads; per-block cost is content-independent",
                by_threads={str(t): dict(value=round(res[t][0], 6), rows=res[t][1], seconds=round(res[t][2], 2))
                            for t in counts},
                cpu_model=model, nproc=nproc,
                threads_note=("the reference's CPU path codes one block at a time (eval_model, "
                              "agents/blkbsdimgcomp_agent.py:565-566 sets one thread): every layer is a GEMV of one "
                              "block's activations, a few hundred microseconds of work, so intra-op threads pay a "
                              "fork/join per layer and their gain depends on how busy the host's other cores are (an "
                              "8-core container: 1 / 4 / 8 threads 0.011 / 0.023 / 0.029 Mpix/s; round 5's box: 16 "
                              "threads below 1); `value` is the fastest thread count measured, up to the job's share "
                              "(OMP_NUM_THREADS; nproc counts the whole machine)"))


def main():
    args = parse_args()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))

    os.environ.setdefault("GPU_MAX_HW_QUEUES", str(args.hw_queues))
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}: launch one process per GPU")
    dist = world > 1
    # test hooks (tests/test_bench_dist_gpu.py runs the N-rank path on a one-GPU box): every rank on one device, and the
    # gloo backend (RCCL refuses two ranks on one GPU).  The driver's runs set neither: one GPU per rank, RCCL.
    local = int(os.environ.get("LBIC_BENCH_DEVICE", local))
    backend = os.environ.get("LBIC_BENCH_BACKEND", "nccl")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    coll_dev = torch.device("cpu") if backend == "gloo" else dev     # where collective operands live
    if dist:
        import torch.distributed as tdist
        if backend == "gloo":
            tdist.init_process_group("gloo")
        else:
            tdist.init_process_group(backend, device_id=dev)

    import types
    from lbic.arch import Arch
    from lbic.layout import image_to_blocks
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.streams import dedicated_streams
    from lbic.weights import synth_state_dict

    B, KS, N, M = CONFIGS[args.config]
    if not args.rate:
        from lbic.weights import rate_for_lambda
        args.rate = rate_for_lambda(CONFIG_LAMBDA[args.config])
    arch = Arch(B, KS, N, M)
    W = args.size
    H = args.height or args.size
    Hb, Wb = H // B, W // B
    cfg = types.SimpleNamespace(block_size=B, KS=list(KS), N=N, M=M, gpu_device=local)
    sd = synth_state_dict(arch, 1337, rate=args.rate)
    n = args.batch

    def make_model():
        m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
        m.load_state_dict(sd)
        m.update(force=True)
        return m

    depth = max(args.depth, 0)
    ndec = max(depth, 2 if args.gang else 1, args.workers - 1, args.team, 1)
    # the encoder's and every decoder's stream first, back to back, so each gets a hardware queue of its own (idle
    # streams created before or between them, only the streams the team schedule uses, or another order moved the
    # encoder's and the decoder's hardware queues and cost up to 10 %: profiles/r03_exp/r03_q_*, r03_bench13_*)
    s_enc, = dedicated_streams(1, dev)
    # (team schedule) the encoder's copy stream right after the encoder's: a hardware queue of its own, not one it would
    # share with the busy team-decoder stream
    s_d2h, = dedicated_streams(1, dev) if args.d2h_stream and args.team else (None,)
    s_decs = dedicated_streams(ndec, dev)
    enc_model = make_model()
    # decoder handles share the encoder handle's packed weights (one copy in the Infinity Cache)
    dec_models = [enc_model.sibling() if args.share_weights else make_model() for _ in range(ndec)]
    if args.enc_lds_floor:
        for m_ in [enc_model] + dec_models:
            m_.set_encoder_lds_floor(args.enc_lds_floor)
    handles = [enc_model] + dec_models
    plock = threading.Lock()

    # two distinct 32-frame sets per rank (batch k codes set k % 2); the gang schedule's encoder passes
    # compress `gang` batches of distinct frames at once
    nsets = max(2, args.gang, args.enc_pass if args.team else 1)
    frames = np.stack([image_to_blocks(np.random.default_rng(rank * n * nsets + k).integers(0, 256, (3, H, W),
                                                                                    dtype=np.uint8)
                                       .astype(np.float32) / 255.0 - 0.5, B) for k in range(n * nsets)])
    xb_all = torch.from_numpy(frames).to(dev)
    del frames

    def frames_of(k):
        s = k % (nsets if args.team and args.enc_pass > 2 else 2)
        return xb_all[s * n:(s + 1) * n]

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(v):
        if dist:
            t = torch.tensor([v], dtype=torch.float64, device=coll_dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            v = float(t.item())
        return v

    enc_acc = dict(on=False, ms=0.0, passes=0)     # HIP-event time of the encoder graphs in the timed region
    # multi-batch encoder passes: the graph as ONE chain of launches (LBC_OPT_ENC_FORK 0; the library's own rule for
    # passes this large), so the graphs' HIP-event wall time over their launches is the launches' average duration
    enc_acc["chain"] = bool(args.team and args.enc_pass > 1)
    enc_model.set_encoder_fork(0 if enc_acc["chain"] else -1)

    def compress_side(ph, xb, model=None, stream=None):
        """GPU compress on the encoder stream; symbols/indexes DMA'd into page-locked host buffers there (for the host
        rANS coder: the reference's coder is host C++).  (Narrowing them to int16 / uint8 and copying on a stream of its
        own moved 2-8 ms per batch off the encoder stream but gained 0.5 %, within noise: profiles/r03_exp.)"""
        model, stream = model or enc_model, stream or s_enc
        t0 = time.perf_counter()
        if s_d2h is not None and stream is s_enc:
            # the copies on their own stream: the encoder stream goes on with the next batch while they run; the device
            # tensors are marked used by the copy stream (the allocator does not hand them out before the copy is
            # done), and the entropy side waits for the copy's event
            with torch.cuda.stream(stream):
                r = model.compress_batch(xb)
                ev = torch.cuda.Event()
                ev.record(stream)
            s_d2h.wait_event(ev)
            with torch.cuda.stream(s_d2h):
                for k in ("symbols", "indexes"):
                    h = torch.empty(r[k].shape, dtype=r[k].dtype, pin_memory=True)
                    h.copy_(r[k], non_blocking=True)
                    r[k].record_stream(s_d2h)
                    r[k] = h
                done = torch.cuda.Event()
                done.record(s_d2h)
            r["d2h_done"] = done
            if not enc_acc["on"]:
                stream.synchronize()      # (untimed / unprofiled passes: one batch at a time, as before)
        else:
            with torch.cuda.stream(stream):
                r = model.compress_batch(xb)
                for k in ("symbols", "indexes"):
                    h = torch.empty(r[k].shape, dtype=r[k].dtype, pin_memory=True)
                    h.copy_(r[k], non_blocking=True)
                    r[k] = h
                stream.synchronize()
        e_ms = model.last_timing()[0] if enc_acc["on"] else 0.0     # (waits for this compress, not for its copy)
        with plock:
            ph["encode"] += time.perf_counter() - t0
            if enc_acc["on"]:
                enc_acc["ms"] += e_ms
                enc_acc["passes"] += 1
        return r

    def split_record(r, e):
        """Batch e (n frames) of a multi-batch compress record."""
        return {kk: (v if kk == "d2h_done" else v[e * n:(e + 1) * n] if v is not None else None) for kk, v in r.items()}

    def entropy_side(r, fmt, ph, model=None):
        t0 = time.perf_counter()
        if r.get("d2h_done") is not None:
            r["d2h_done"].synchronize()
        st = (model or enc_model).entropy_encode(r["symbols"], r["indexes"], fmt=fmt, Hb=Hb, Wb=Wb)
        with plock:
            ph["entropy"] += time.perf_counter() - t0
        return st

    def decode_side(i, st, fmt, ph, model=None, stream=None):
        model, stream = model or dec_models[i], stream or s_decs[i]
        t0 = time.perf_counter()
        with torch.cuda.stream(stream):
            z = model.decompress_batch(st, Hb, Wb, fmt=fmt)
            stream.synchronize()
        with plock:
            ph["decode"] += time.perf_counter() - t0
        return z

    def collect_stats():
        ks = {}
        for m_ in handles:
            for name, st_ in (m_.profile_end() or {}).items():
                acc = ks.setdefault(name, {k: 0.0 for k in st_})
                for k_ in st_:
                    acc[k_] += st_[k_]
        return ks

    team_acc = dict(launches=0, ms=0.0, bytes=0.0, flops=0.0, steps=0, plain=[], timeouts=0, windows=[], enc_done=0.0,
                    modes=[])

    def pipeline(steps, depth, fmt="reference", gang=1, prof=False, label="", base=0, workers=0, team=0, tbatches=0,
                 enc_pass=0):
        """`steps` batches through the pipeline, all inside the timed region: this thread compresses batch k
        (or `gang` batches in one wavefront pass) while a helper thread entropy codes the previous one and
        `depth` decoder threads each decode `gang` queued batches per raster pass (their own handles and
        streams; ctypes drops the GIL).  depth 0: encode, entropy, decode one after another.
        Returns (seconds, phase seconds, last decoded (record, streams, zhat), kernel stats)."""
        ph = dict(encode=0.0, entropy=0.0, decode=0.0)
        if prof:
            for m_ in handles:
                m_.profile_begin(sample_every)
            enc_acc.update(on=True, ms=0.0, passes=0)
            # marker kernels (at::cuda spin_kernel) around the timed region: tools/kstats_summary.py restricts a
            # rocprofv3 kernel trace of this command to the dispatches between them
            torch.cuda._sleep(1000)
        barrier()
        t0 = time.perf_counter()
        done = dict(count=0, last=None)      # only the latest batch is kept (its pinned / device buffers)

        def finish(k_, r_, st_, z_):
            # the latest batch with a record (the team schedule keeps the record of the last batch only)
            with plock:
                done["count"] += 1
                cur = done["last"]
                if cur is None or ((r_ is not None) == (cur[1] is not None) and k_ > cur[0]) or \
                        (r_ is not None and cur[1] is None):
                    done["last"] = (k_, r_, st_, z_)
        if team:
            # the encoder handle compresses batch after batch on its stream (host rANS on helper threads); a decoder
            # thread takes the encoded batches in groups of `team` and decodes each group in ONE persistent launch
            # (one team of workgroups per batch) on its own stream, beside the encoder's next batches
            from concurrent.futures import ThreadPoolExecutor
            from lbic.model import decompress_teams
            dq = queue.Queue(maxsize=2 * team)
            if prof:
                for kk in team_acc:
                    team_acc[kk] = [] if kk in ("plain", "windows", "modes") else 0
                team_acc["hw"] = Hb * Wb
                to0 = dec_models[0].team_stats()["timeout_fallbacks"]
            errs = []

            # group sizes (batches per launch, up to team x --team-batches): with --team-groups last-full (default) a
            # partial group comes FIRST, so the launch that runs alone after the last encode (the drain) is a full one
            # and the first launch starts earlier
            tb = tbatches or args.team_batches
            sizes = team_group_sizes(steps, team, tb, args.team_groups,
                                     args.team_sizes if args.team_sizes and steps == args.steps else "",
                                     args.first_team_batches if not tbatches else 0, len(dec_models))

            def first_size(teams):
                if args.first_team_size >= 0:
                    return args.first_team_size
                return 12 if teams <= 8 else 0

            def team_decoder():
                pend = []
                gi = 0
                try:
                    while True:
                        it = dq.get()
                        if it is not None:
                            pend.append(it)
                        if pend and (it is None or len(pend) == sizes[min(gi, len(sizes) - 1)]):
                            gi += 1
                            t0_ = time.perf_counter()
                            sts = [f_.result() for (_, _, f_) in pend]
                            last = gi == len(sizes)
                            sd_ = s_decs[0]
                            # teams of tb_ batches (their images side by side: a team of 2 x 32 images); a group of
                            # an odd count: one batch per team
                            tb_ = args.first_team_batches if gi == 1 and args.first_team_batches and not tbatches else tb
                            tb_ = tb_ if len(pend) % tb_ == 0 else 1     # (team_group_sizes keeps len(pend) <= team)
                            tsts = [[s_ for st_ in sts[i:i + tb_] for s_ in st_] for i in range(0, len(sts), tb_)]
                            with torch.cuda.stream(sd_):
                                # (two workgroups per CU for the last launch measured slower:
                                # profiles/r02_exp/team_two_per_cu.txt)
                                zt = decompress_teams(dec_models[:len(tsts)], tsts, Hb, Wb,
                                                      wg_per_cu=args.drain_wg_per_cu if last else 1,
                                                      team_size=first_size(len(tsts)) if gi == 1 and not last else 0)
                                sd_.synchronize()
                            zs = [z_[e * n:(e + 1) * n] for z_ in zt for e in range(tb_)]
                            with plock:
                                ph["decode"] += time.perf_counter() - t0_
                            if prof:
                                st_ = dec_models[0].team_stats()
                                team_acc["launches"] += 1
                                team_acc["ms"] += st_["launch_ms"]
                                team_acc["bytes"] += st_["bytes"]
                                team_acc["flops"] += st_["flops"]
                                team_acc["steps"] += len(pend) * Hb * Wb
                                team_acc["plain"].append(st_["plain"])
                                team_acc["modes"].append(st_["mode"])
                                team_acc["timeouts"] = st_["timeout_fallbacks"] - to0
                                team_acc["windows"].append([round(t0_ - t0, 3), round(time.perf_counter() - t0, 3),
                                                            len(pend), len(tsts)])
                            for (k_, r_, _), st_, z_ in zip(pend, sts, zs):
                                finish(k_, r_, st_, z_)
                            pend = []
                        if it is None:
                            return
                except BaseException as e:    # surfaced by the encoder thread below
                    errs.append(e)
                    while dq.get() is not None:
                        pass

            dth = threading.Thread(target=team_decoder)
            dth.start()
            with ThreadPoolExecutor(max_workers=4) as ex:
                k = 0
                while k < steps:
                    P_ = enc_pass or args.enc_pass
                    g = min(P_, steps - k)
                    if P_ == 1 or (base + k) % P_:
                        g = 1
                        rs_ = [compress_side(ph, frames_of(base + k))]
                    else:
                        # batches k .. k + P - 1 = frame sets 0 .. P - 1 (contiguous in xb_all): one wavefront pass.  A
                        # short last group is coded in a full pass as well (the missing partners' codes are dropped):
                        # the encoder graph keeps one frame count, so no pass re-captures it
                        rr_ = compress_side(ph, xb_all[:P_ * n])
                        rs_ = [split_record(rr_, e) for e in range(g)]
                        del rr_
                    for e, r_ in enumerate(rs_):
                        f_ = ex.submit(entropy_side, r_, fmt, ph)
                        # only the last batch keeps its record (zhat, symbols) for the quality check
                        dq.put((base + k + e, r_ if k + e == steps - 1 else None, f_))
                    del rs_, r_
                    k += g
                if prof:
                    team_acc["enc_done"] = round(time.perf_counter() - t0, 3)
                dq.put(None)
                dth.join()
            if errs:
                raise errs[0]
        elif workers:
            # every worker (its own handle + stream) takes the next batch and compresses, entropy codes and decodes it
            wk = list(zip([enc_model] + dec_models, [s_enc] + s_decs))[:workers]
            nxt = dict(k=0)
            nlock = threading.Lock()

            from concurrent.futures import ThreadPoolExecutor

            def worker(wi):
                # the host rANS of batch k runs on a helper thread while this worker's stream compresses its next
                # batch, so the stream does not idle through it; then batch k is decoded
                m_, s_ = wk[wi]
                prev = None                   # (k, record, future of its streams)
                with ThreadPoolExecutor(max_workers=1) as ex:
                    while True:
                        with nlock:
                            k = nxt["k"]
                            nxt["k"] += 1
                        cur = None
                        if k < steps:
                            r_ = compress_side(ph, frames_of(base + k), m_, s_)
                            cur = (k, r_, ex.submit(entropy_side, r_, fmt, ph, m_))
                        if prev is not None:
                            k_, r_, f_ = prev
                            st_ = f_.result()
                            finish(base + k_, r_, st_, decode_side(wi, st_, fmt, ph, m_, s_))
                        if cur is None:
                            return
                        prev = cur

            ths = [threading.Thread(target=worker, args=(i,)) for i in range(workers)]
            for th in ths:
                th.start()
            for th in ths:
                th.join()
        elif depth == 0:
            for k in range(steps):
                r = compress_side(ph, frames_of(base + k))
                st = entropy_side(r, fmt, ph)
                finish(base + k, r, st, decode_side(0, st, fmt, ph))
        else:
            q = queue.Queue(maxsize=depth * gang)      # encoded batches waiting for a decoder
            eq = queue.Queue(maxsize=1)                # compressed batches waiting for the host rANS
            glock = threading.Lock()

            def decoder(i):
                while True:
                    items, end = [], False
                    with glock:                        # one decoder gathers its whole gang
                        while len(items) < gang:
                            it = q.get()
                            if it is None:
                                end = True
                                break
                            items.append(it)
                    if items:
                        z_ = decode_side(i, [b for (_, _, st_) in items for b in st_], fmt, ph)
                        for j, (k_, r_, st_) in enumerate(items):
                            finish(k_, r_, st_, z_[j * n:(j + 1) * n])
                    if end:
                        q.put(None)
                        return

            def entropy_worker():
                while True:
                    it = eq.get()
                    if it is None:
                        q.put(None)
                        return
                    for k_, r_ in it:
                        q.put((k_, r_, entropy_side(r_, fmt, ph)))

            ths = [threading.Thread(target=decoder, args=(i,)) for i in range(depth)]
            eth = threading.Thread(target=entropy_worker)
            for th in ths + [eth]:
                th.start()
            for k in range(0, steps, gang):
                g = min(gang, steps - k)
                if g == 1:
                    eq.put([(base + k, compress_side(ph, frames_of(base + k)))])
                else:       # one wavefront pass over g batches of distinct frames
                    r = compress_side(ph, xb_all[:g * n])
                    eq.put([(base + k + e, split_record(r, e)) for e in range(g)])
            eq.put(None)
            eth.join()
            for th in ths:
                th.join()
        barrier()
        local_dt = time.perf_counter() - t0
        dt = max_over_ranks(local_dt)
        if prof:
            enc_acc["on"] = False
            torch.cuda._sleep(1000)
            torch.cuda.synchronize(dev)
        ks = collect_stats() if prof else None
        if label:
            log(f"[rank {rank}] {label}: {steps} batches in {dt:.2f} s (this rank {local_dt:.4f} s)")
        if done["count"] != steps:
            raise RuntimeError(f"{label}: {done['count']} of {steps} batches decoded")
        return dt, ph, done["last"][1:], ks

    def summary(dt, ph, k, **extra):
        return dict(value=round(world * n * H * W / (dt / k) / 1e6, 4), ms_per_step=round(dt / k * 1e3, 2),
                    steps=k, phases_ms_per_step={kk: round(v / k * 1e3, 2) for kk, v in ph.items()}, **extra)

    # sampling is part of the captured graphs: enable it before the first capture.  The team schedule: its decode is
    # one persistent launch (HIP events); the encoder graph is timed by HIP events AND every --enc-sample-every-th
    # wavefront step's launches carry in-kernel stamps (a launch's own duration: the graph's two branches overlap)
    sample_every = args.enc_sample_every if args.team else args.sample_every
    for m_ in handles:
        m_.profile_begin(sample_every)
    if args.encode_only:      # e.g. rocprofv3 --pmc on the encoder's launch shapes
        for i in range(args.encode_only):
            compress_side(dict(encode=0.0, entropy=0.0, decode=0.0), frames_of(i))
            log(f"[rank {rank}] encoder pass {i + 1}/{args.encode_only} done")
        return

    # warmup: every decoder handle builds its row graphs, then `warmup` batches through the pipeline
    scratch = dict(encode=0.0, entropy=0.0, decode=0.0)
    if args.team and args.enc_pass > 1:
        compress_side(scratch, xb_all[:args.enc_pass * n])       # the multi-batch encoder graph (captured once)
    r0 = compress_side(scratch, frames_of(0))
    st0 = entropy_side(r0, "reference", scratch)
    if not args.team:
        for i in range(len(dec_models)):
            decode_side(i, st0, "reference", scratch)
    if args.workers and not args.team:       # every worker handle encodes too: build its encoder graph
        for m_, s_ in list(zip(dec_models, s_decs))[:args.workers - 1]:
            compress_side(scratch, frames_of(0), m_, s_)
    if args.warmup > 0:
        pipeline(args.warmup, max(depth, 1) if depth else 0, label="warmup", workers=args.workers, team=args.team)
    if args.team and (args.team_batches > 1 or args.team > args.warmup):
        # every decoder handle's workspace sized for a team's images and the full launch's team program recorded before
        # the timed region (one untimed launch of full teams on the warmup batch's streams)
        from lbic.model import decompress_teams
        with torch.cuda.stream(s_decs[0]):
            decompress_teams(dec_models[:args.team], [st0 * args.team_batches] * args.team, Hb, Wb)
            s_decs[0].synchronize()

    # ---- headline: the reference bitstream format, one 32-frame batch per decode pass
    dt, phase, (r, streams, z), kstats = pipeline(args.steps, depth, prof=True, label="headline", workers=args.workers,
                                                  team=args.team)

    side = {}
    if args.side_steps > 0 and args.team and args.enc_pass > 1:
        # the same schedule with every 32-frame batch encoded as its own wavefront pass (the round-5 headline's encoder,
        # its graph forked as the library's default rule does for passes this small; captured before the leg)
        enc_model.set_encoder_fork(-1)
        entropy_side(compress_side(dict(encode=0.0, entropy=0.0, decode=0.0), frames_of(0)), "reference",
                     dict(encode=0.0, entropy=0.0, decode=0.0))
        d_, p_, _, _ = pipeline(args.steps, depth, label="one batch per encode pass", team=args.team, enc_pass=1)
        side["one_batch_per_encode_pass"] = summary(d_, p_, args.steps, frames_per_encode_pass=n)
        enc_model.set_encoder_fork(0)
    if args.side_steps > 0 and args.team == 16 and args.team_batches == 1:
        # the round-4 geometry beside it: 8 teams per launch, one per XCD (each a whole XCD's CUs), same batches (the
        # headline's encoder graph captured again before the leg: a handle keeps one)
        if args.enc_pass > 1:
            compress_side(dict(encode=0.0, entropy=0.0, decode=0.0), xb_all[:args.enc_pass * n])
        d_, p_, _, _ = pipeline(args.steps, depth, label="8 teams per launch", team=8)
        side["eight_teams_per_launch"] = summary(d_, p_, args.steps, frames_in_flight_per_decode_pass=n,
                                                 decode_passes_in_flight=8)
    if args.side_steps > 0 and (depth != 1 or args.team or args.workers):
        d_, p_, _, _ = pipeline(args.side_steps, 1, label="one decode in flight")
        side["one_decode_in_flight"] = summary(d_, p_, args.side_steps, frames_in_flight_per_decode_pass=n,
                                               decode_passes_in_flight=1)
    if args.side_steps > 0 and (depth != 0 or args.team or args.workers):
        d_, p_, _, _ = pipeline(args.side_steps, 0, label="serial")
        side["serial_schedule"] = summary(d_, p_, args.side_steps)
    gang_s = None
    if args.gang > 1 and depth >= 1:
        gsteps = 2 * args.gang                    # one gang pass per decoder handle, both in the region
        # (the decoders' graphs for gang x n streams are built by an untimed pass first)
        pipeline(2 * args.gang, 2, gang=args.gang, label="gang warmup")
        d_, p_, _, _ = pipeline(gsteps, 2, gang=args.gang, label="gang")
        gang_s = summary(d_, p_, gsteps, frames_in_flight_per_decode_pass=args.gang * n, decode_passes_in_flight=2,
                         batches_per_encode_pass=args.gang,
                         note="not the headline: a raster pass over several queued batches (more frames in flight "
                              "than the batch-32 config)")
    sub = None
    if args.substream_steps > 0:
        pipeline(max(depth, 1), max(depth, 1), fmt="rows", label="rows warmup")
        d_, p_, (rs, ss, zs), _ = pipeline(args.substream_steps, max(depth, 1), fmt="rows", label="rows")
        sub = summary(d_, p_, args.substream_steps,
                      bpp=round(float(np.mean([len(b) * 8.0 / (H * W) for b in ss])), 5),
                      enc_dec_bit_exact=bool(torch.equal(zs, rs["zhat"])),
                      note="opt-in per-block-row sub-stream container (not the reference bitstream)")

    # ---- quality of the last decoded batch (outside the timed region) + parity against the reference's
    #      full-frame fixture (tests/golden), when this is its configuration
    bit_exact = bool(torch.equal(z, r["zhat"]))
    xq = frames_of(max(0, args.steps - 1))
    sse = ((z - xq) ** 2).double().sum(dim=(1, 2, 3))
    rec = torch.stack([torch.tensor([float(len(s)) for s in streams], dtype=torch.float64, device=dev), sse,
                       torch.full((n,), float(H * W * 3), dtype=torch.float64, device=dev)], dim=1)
    rec, bit_exact = gather_records(rec.to(coll_dev), bit_exact, dist)
    rec = rec.cpu().numpy()
    bpp = float(np.mean(rec[:, 0] * 8.0 / (H * W)))
    psnr = float(np.mean(-10 * np.log10(rec[:, 1] / rec[:, 2])))
    vs_ref = tq = per_img = None
    if rank == 0:
        vs_ref = compare_full_frame_fixture(enc_model, args, arch, dev)
        if args.side_steps > 0:
            tq = transform_quality(arch, cfg, dev, H, W)
        if args.per_image:
            per_img = per_image_timing(enc_model, dec_models, arch, H, W, dev)

    if rank != 0:
        if dist:
            torch.distributed.destroy_process_group()
        return

    ms_step = dt / args.steps * 1e3
    value = world * n * H * W / (dt / args.steps) / 1e6

    headline_shape = (args.config, H, W, n) == ("B8_lowrate", 768, 768, 32)
    roof, kernels = roofline(kstats, dt, team_acc if args.team else None, enc_acc if args.team else None, args.steps,
                             cfg_key=None if headline_shape else args.config)
    mac_enc, mac_dec = arch.live_macs_per_block()
    step_flops = 2.0 * (mac_enc + mac_dec) * Hb * Wb * n
    cpu = None
    if args.cpu_budget > 0 and world == 1:
        cpu = cpu_baseline(arch, sd, H, W, args.cpu_budget)

    tb_cfg = args.team_batches if args.team else 1
    first_teams = 0
    if args.team and team_acc["windows"] and len(team_acc["windows"]) > 1:
        first_teams = team_acc["windows"][0][3]          # teams of the first launch (the one beside the encoder)
    fts_used = args.first_team_size if args.first_team_size >= 0 else (12 if first_teams <= 8 else 0)
    enc_desc = (f"{args.enc_pass} batches encoded in one {args.enc_pass * n}-frame wavefront pass" if args.team and
                args.enc_pass > 1 else f"each batch encoded as its own {n}-frame wavefront pass")
    out = {
        "metric": METRIC if (args.config, H, W) == ("B8_lowrate", 768, 768) else
        f"Mpixels/s encode+decode, {args.config} N{N}M{M}, {W}×{H}", "value": round(value, 4), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": f"synthetic: seeded uint8 noise frames, seeded synthetic weights at the '{args.rate}' operating point "
                "(no checkpoints / Kodak offline)",
        "config": {"workload": f"{args.config} N{N}M{M}, batches of {n} synthetic {H}x{W} frames per GPU, encode+decode "
                               f"in the reference bitstream format (one raster rANS stream per image); "
                               + ((f"{enc_desc}, each batch entropy coded and decoded as its own "
                                   f"{n}-frame raster pass by one team of workgroups; up to {args.team} passes in one "
                                   "persistent launch (one team per XCD up to 8, two per XCD beyond)"
                                   if tb_cfg == 1 else
                                   f"{enc_desc}; decode: {tb_cfg} batches per "
                                   f"team of workgroups ({n * tb_cfg} images per team side by side), up to {args.team} "
                                   "teams per launch")
                                  + (f"; the first launch (beside the encoder's next batches: {first_teams} teams) on "
                                     + (f"{first_wg_per_xcd(first_teams, fts_used)} of every busy XCD's 32 CUs" if fts_used
                                        else "every CU")
                                     if first_teams else "") if args.team else
                                  f"each decode pass decodes one {n}-frame batch ({n} frames in flight per pass), "
                                  f"up to {args.workers} passes in flight (one per worker)" if args.workers else
                                  f"each decode pass decodes one {n}-frame batch ({n} frames in flight per pass), "
                                  f"{depth} pass(es) in flight beside the encoder"),
                   "batch_per_gpu": n, "frame": [H, W], "parallelism": f"images sharded over {world} GPU(s)",
                   "global_batch": n * world, "frames_in_flight_per_decode_pass": n * (tb_cfg if args.team else 1),
                   "decode_passes_in_flight": args.team or args.workers or depth,
                   "frames_per_encode_pass": n * (args.enc_pass if args.team else 1),
                   "schedule": (f"team: one encoder handle (own HIP stream) compresses batch after batch, host rANS on "
                                f"helper threads; every {args.team * tb_cfg} encoded batches (the first group: the "
                                "remainder) are decoded by ONE persistent k_dec_team launch on a second stream "
                                f"(lbc_decode_team: a team of workgroups per {'batch' if tb_cfg == 1 else f'{tb_cfg} batches'}, "
                                "team barriers instead of kernel boundaries), beside the next encodes"
                                if args.team else
                                f"workers: {args.workers} codec handles on one weight set, each with its own HIP stream "
                                "and host thread, take the batches in turn and compress, entropy code (host rANS) and "
                                "decode each whole batch" if args.workers else
                                "serial: encode, entropy, decode per batch" if depth == 0 else
                                f"pipeline: encoder (own handle + stream) compresses batch k+1 while {depth} decoder "
                                "handle(s) (own handle + stream each) decode earlier batches, host rANS on a helper "
                                "thread")
                   + "; the timed region holds the compress and decompress of the same batches, fill and drain "
                     "included"},
        "roofline": roof, "cpu_baseline": cpu,
        "quality": {"rate_point": args.rate, "bpp": round(bpp, 5), "psnr_db": round(psnr, 3),
                    "enc_dec_bit_exact": bit_exact, "images_gathered": int(rec.shape[0]), "vs_ref": vs_ref,
                    "transform_point": tq},
        "per_image": per_img,
        "phases_ms_per_step": {k: round(v / args.steps * 1e3, 2) for k, v in phase.items()},
        "step_algorithmic_tflop": round(step_flops / 1e12, 3),
        "step_mfma_frac": round(step_flops / (dt / args.steps) / (PEAK_FP32_TFLOPS * 1e12), 5),
        "kernels": kernels,
        **side,
        "gang_schedule": gang_s,
        "substream_format": sub,
    }
    print(json.dumps(out), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


def gather_records(rec, ok, dist):
    """The run's only data collective: every rank's per-image [bytes, SSE, n_px] records all-gathered (RCCL over
    xGMI on the GPU box, gloo in the CPU test) and the encoder/decoder agreement MIN-reduced."""
    import torch
    if not dist:
        return rec, ok
    import torch.distributed as tdist
    allrec = [torch.empty_like(rec) for _ in range(tdist.get_world_size())]
    tdist.all_gather(allrec, rec)
    flag = torch.tensor([1.0 if ok else 0.0], dtype=torch.float64, device=rec.device)
    tdist.all_reduce(flag, op=tdist.ReduceOp.MIN)
    return torch.cat(allrec), bool(flag.item() == 1.0)


def roofline(kstats, dt, team=None, enc=None, steps=0, cfg_key=None):
    """Dominant kernel family against its roofline.  Dominance = wall occupancy in the timed region, i.e. the time
    during which the family has a launch running, overlap with OTHER families allowed but never counted twice within
    one family: for the team decoder the summed durations of its launches (one at a time, HIP events around each), for
    the encoder's GEMM family the summed wall time of the encoder graphs (HIP events around each graph: its forked
    branches run two of its launches at once, so the launches' summed durations exceed the graph's wall time and are
    not its occupancy).  Graph-launched kernels: per-launch durations from the in-kernel timing stamps of the sampled
    launches executed in the timed region (lbc_profile_*; earliest workgroup start -> latest end, what a dispatch trace
    such as rocprofv3 --kernel-trace reports); the encoder family is also reported as an aggregate (its algorithmic
    FLOPs over the encoder graphs' wall time).  The team decoder: algorithmic bytes / FLOPs per launch from the library
    (lbc_team_stats)."""
    kernels, fam = {}, {}
    if enc is not None and kstats:
        egm = "k_gemm_t" if "k_gemm_t" in kstats else "k_gemm"       # lbc_profile names the family by its kernel
        efam = (egm, "k_gemm", "k_gemm_s")      # every launch of the encoder graphs (k_gemm: the narrow-N layers)
        n_all = sum(s["total_launches"] for k_, s in kstats.items() if k_ in efam)
        sg = kstats.get(egm, {})
        if n_all and enc["ms"] > 0:
            wall = enc["ms"] / n_all
            tf = sum(s["total_flops"] for k_, s in kstats.items() if k_ in efam)
            tb = sum(s["total_bytes"] for k_, s in kstats.items() if k_ in efam)
            agg = dict(encoder_wall_s=round(enc["ms"] / 1e3, 4), encoder_graphs=enc["passes"],
                       tflop=round(tf / 1e12, 4), achieved_tflops=round(tf / (enc["ms"] / 1e3) / 1e12, 3),
                       frac=round(tf / (enc["ms"] / 1e3) / (PEAK_FP32_TFLOPS * 1e12), 5),
                       note=f"every launch of the encoder graphs ({', '.join(k_ for k_ in efam if k_ in kstats)}): "
                            "algorithmic FLOPs / the graphs' wall time")
            if sg.get("launches") and enc.get("chain") and n_all == sg["total_launches"]:
                # one chain of launches (no fork): HIP events around the graphs / the launches = a launch's average
                # duration incl. the dependent-launch gap (an upper bound on the kernel time); the in-kernel stamps
                # (earliest workgroup start -> latest end over the XCDs' clocks) are reported beside it
                per = sg["total_ms"] / sg["launches"]
                n_k = int(sg["total_launches"])
                kernels[egm] = dict(launches_sampled=int(sg["launches"]), launches_total=n_k,
                                    avg_span_us=round(wall * 1e3, 3), avg_launch_us=round(wall * 1e3, 3),
                                    stamped_span_us=round(per * 1e3, 3), wall_us_per_launch=round(wall * 1e3, 3),
                                    wall_occupancy_s=round(enc["ms"] / 1e3, 4),
                                    summed_launch_s=round(enc["ms"] / 1e3, 4), aggregate=agg,
                                    timing=f"HIP events around the encoder graphs (one chain of {n_k} launches: "
                                           f"{enc['ms'] / 1e3:.3f} s over {enc['passes']} graphs) / their launches; "
                                           f"in-kernel stamps of every sampled launch: stamped_span_us")
                fam[egm] = (tf / n_all, tb / n_all)
            elif sg.get("launches"):
                per = sg["total_ms"] / sg["launches"]
                n_k = int(sg["total_launches"])
                kernels[egm] = dict(launches_sampled=int(sg["launches"]), launches_total=n_k,
                                    avg_span_us=round(per * 1e3, 3), avg_launch_us=round(per * 1e3, 3),
                                    wall_us_per_launch=round(wall * 1e3, 3),
                                    wall_occupancy_s=round(enc["ms"] / 1e3, 4),
                                    summed_launch_s=round(per * n_k / 1e3, 4), aggregate=agg,
                                    timing=f"in-kernel stamps of the sampled {egm} launches (earliest workgroup start -> "
                                           "latest end); occupancy = HIP events around the encoder graphs "
                                           f"({enc['ms'] / 1e3:.3f} s over {enc['passes']} graphs)")
                fam[egm] = (sg["flops"] / sg["launches"], sg["bytes"] / sg["launches"])
            else:
                kernels[egm] = dict(launches_sampled=0, launches_total=int(n_all), avg_span_us=round(wall * 1e3, 3),
                                    avg_launch_us=round(wall * 1e3, 3), wall_us_per_launch=round(wall * 1e3, 3),
                                    wall_occupancy_s=round(enc["ms"] / 1e3, 4), aggregate=agg,
                                    timing=f"HIP events around {enc['passes']} encoder graphs / their launches "
                                           f"({egm} + k_gemm_s ramp steps; the forked branches overlap, so this "
                                           "understates a launch's own duration)")
                fam[egm] = (tf / n_all, tb / n_all)
        kstats = {}
    for name, s in (kstats or {}).items():
        span = s["total_ms"] / max(s["launches"], 1)
        per = s["total_ms_chain"] / s["launches_chain"] if s["launches_chain"] else span
        kernels[name] = dict(launches_sampled=int(s["launches"]), launches_total=int(s["total_launches"]),
                             avg_span_us=round(span * 1e3, 3), avg_launch_us=round(per * 1e3, 3),
                             wall_occupancy_s=round(per * s["total_launches"] / 1e3, 4))
        fam[name] = (s["flops"] / max(s["launches"], 1), s["bytes"] / max(s["launches"], 1))
    if team and team["launches"]:
        per = team["ms"] / team["launches"]
        kernels["k_dec_team"] = dict(launches_sampled=team["launches"], launches_total=team["launches"],
                                     avg_span_us=round(per * 1e3, 3), avg_launch_us=round(per * 1e3, 3),
                                     wall_occupancy_s=round(team["ms"] / 1e3, 4),
                                     plain_handoffs=team["plain"],
                                     barrier_timeout_fallbacks=team["timeouts"],
                                     launch_windows_s=team["windows"], encoder_done_s=team["enc_done"],
                                     modes=team.get("modes", []),
                                     batches_per_launch=round(team["steps"] / team["launches"] / team["hw"], 3),
                                     batch_decode_latency_ms=round(per, 3),
                                     launch_ms_per_batch=round(team["ms"] * team["hw"] / team["steps"], 3),
                                     timing="HIP events around each launch")
        fam["k_dec_team"] = (team["flops"] / team["launches"], team["bytes"] / team["launches"])
    if not kernels:
        return None, {}
    dom = max(kernels, key=lambda k: kernels[k]["wall_occupancy_s"])
    if not fam[dom][1]:
        return None, kernels
    ridge = PEAK_FP32_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)

    def bound_of(name):
        fl_, by_ = fam[name]
        s_ = kernels[name]["avg_launch_us"] * 1e-6
        if fl_ > 0 and by_ and fl_ / by_ >= ridge:
            return fl_ / s_ / 1e12, PEAK_FP32_TFLOPS, "TFLOP/s", "mfma"
        return by_ / s_ / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
    traffic_db = {}
    tfile = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    if os.path.exists(tfile):       # rocprofv3 PMC passes (tools/pmc_round.sh)
        with open(tfile) as fh:
            traffic_db = json.load(fh)

    def traffic_of(name):
        # counters taken at this configuration's own launch shapes (tools/pmc_configs.sh) when it is not the headline's
        pm = traffic_db.get("configs", {}).get(cfg_key, {}).get(name, {}) if cfg_key else traffic_db.get(name, {})
        if name == "k_dec_team" and team and "hbm_bytes_per_batch_step" in pm:
            # (counters at the headline's team shape; team["steps"] counts 32-frame batch raster steps)
            return round(pm["hbm_bytes_per_batch_step"] * team["steps"] / team["launches"]), pm.get("source")
        if "hbm_bytes_per_dispatch" in pm:
            return round(pm["hbm_bytes_per_dispatch"]), pm.get("source")
        return None, None
    per_kernel = {}
    for name in kernels:
        if name in fam and fam[name][1]:
            a_, p_, u_, b_ = bound_of(name)
            tr_, src_ = traffic_of(name)
            per_kernel[name] = dict(bound=b_, achieved=round(a_, 4), peak=p_, unit=u_, frac=round(a_ / p_, 5),
                                    avg_launch_us=kernels[name]["avg_launch_us"],
                                    wall_occupancy_s=kernels[name]["wall_occupancy_s"],
                                    algorithmic_per_launch=dict(flops=round(fam[name][0]), bytes=round(fam[name][1])),
                                    traffic=tr_, traffic_source=src_)
            if "aggregate" in kernels[name]:
                per_kernel[name]["aggregate"] = kernels[name]["aggregate"]
    fl, by = fam[dom]
    ai = fl / by if by else float("inf")
    ach, peak, unit, bound = bound_of(dom)
    traffic, tsrc = traffic_of(dom)
    roof = dict(kernel=dom, bound=bound, achieved=round(ach, 4), peak=peak, unit=unit, frac=round(ach / peak, 5),
                traffic=traffic, traffic_source=tsrc,
                avg_launch_us=kernels[dom]["avg_launch_us"], avg_span_us=kernels[dom]["avg_span_us"],
                algorithmic_per_launch=dict(flops=round(fl), bytes=round(by)), arithmetic_intensity=round(ai, 2),
                wall_occupancy_s=kernels[dom]["wall_occupancy_s"],
                wall_occupancy_ms_per_step=round(kernels[dom]["wall_occupancy_s"] * 1e3 / steps, 3) if steps else None,
                per_kernel=per_kernel,
                dominant_rule="largest wall occupancy in the timed region: the time the family has a launch running "
                              "(team decoder: summed launch durations; encoder GEMMs: the encoder graphs' wall time)")
    return roof, kernels


def per_image_timing(enc_model, dec_models, arch, H, W, dev, reps=3):
    """The reference's per-image timed region (eval_model, agents/blkbsdimgcomp_agent.py:591-599): compress() of ONE
    frame (batch 1: GPU wavefront + host rANS) and decompress() of its bitstream, each bracketed by
    torch.cuda.synchronize() and timed on the host clock as the reference does, through the reference interface
    (lbic.model: compress / decompress -> lbc_encode + lbc_rans_encode / lbc_decode).  Beside it, the same bitstream
    through a team launch of one batch (decompress_teams, T = 1).  Median of `reps` (after one untimed pass)."""
    import numpy as np
    import torch
    from lbic.layout import image_to_blocks
    from lbic.model import decompress_teams
    img = np.random.default_rng(12345).integers(0, 256, (3, H, W), dtype=np.uint8).astype(np.float32) / 255.0 - 0.5
    xb = torch.from_numpy(image_to_blocks(img, arch.B)).to(dev)
    x = xb.permute(2, 0, 1)[None].contiguous()            # [1, 3B^2, Hb, Wb], the reference's layout
    lru = [arch.lru] * 3
    enc, dec, team = [], [], []
    for k in range(reps + 1):
        torch.cuda.synchronize(dev)
        t0 = time.time()
        bs, zhat = enc_model.compress(x, lru, arch.M)
        torch.cuda.synchronize(dev)
        t1 = time.time()
        z = dec_models[0].decompress(bs, lru, x.shape, arch.M, dev)
        torch.cuda.synchronize(dev)
        t2 = time.time()
        zt = decompress_teams(dec_models[:1], [[bs]], H // arch.B, W // arch.B)[0]
        torch.cuda.synchronize(dev)
        t3 = time.time()
        if k:
            enc.append(t1 - t0)
            dec.append(t2 - t1)
            team.append(t3 - t2)
        exact = bool(torch.equal(z, zhat)) and bool(torch.equal(zt[0], zhat[0].permute(1, 2, 0)))
    med = lambda v: round(float(np.median(v)) * 1e3, 2)
    return dict(frame=[H, W], bpp=round(len(bs) * 8.0 / (H * W), 5), enc_ms=med(enc), dec_ms=med(dec),
                dec_team_ms=med(team), enc_dec_bit_exact=exact, dec_path=dec_models[0].decode_path(),
                dec_team_mode=dec_models[0].team_stats()["mode"],
                note="eval_model's per-image Enc/DecTime (batch 1, host clock around synchronize): compress() = "
                     "lbc_encode + host rANS, decompress() = lbc_decode (one image: the single-image decoder k_dec_one "
                     "where it applies -- dec_path -- else the raster row graphs); dec_team_ms: the same stream through "
                     "decompress_teams with one batch of one image (lbc_decode_team hands a single image to lbc_decode: "
                     "dec_team_mode 'one')")


def transform_quality(arch, cfg, dev, H, W, n=4):
    """Quality at a working operating point (outside the timed region): the network with transform-codec weights
    (lbic.weights.transform_state_dict: block DCT, frequency-weighted steps, no prediction) codes n structured
    synthetic frames (smooth_frame) through the same library path -- compress, host rANS, GPU decode.  The
    headline's weights are random at the config's rate, so its own PSNR carries no information; this one does."""
    import numpy as np
    import torch
    from lbic.layout import image_to_blocks
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.weights import TRANSFORM_STEP, smooth_frame, transform_state_dict
    try:
        sd = transform_state_dict(arch)
    except ValueError as e:
        return {"skipped": str(e)}
    m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
    m.load_state_dict(sd)
    m.update(force=True)
    xb = torch.from_numpy(np.stack([image_to_blocks(smooth_frame(100 + i, H, W).astype(np.float32) / 255.0 - 0.5,
                                                    arch.B) for i in range(n)])).to(dev)
    r = m.compress_batch(xb)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    z = m.decompress_batch(st, H // arch.B, W // arch.B)
    mse = ((z - xb) ** 2).double().mean(dim=(1, 2, 3)).cpu().numpy()
    out = {"weights": f"transform_state_dict (block DCT, step {TRANSFORM_STEP}, {arch.M} coefficients)",
           "frames": f"{n} smooth_frame synthetic {H}x{W}",
           "bpp": round(float(np.mean([len(s) * 8.0 / (H * W) for s in st])), 5),
           "psnr_db": round(float(np.mean(-10 * np.log10(mse))), 3),
           "enc_dec_bit_exact": bool(torch.equal(z, r["zhat"]))}
    return out


def compare_full_frame_fixture(model, args, arch, dev):
    """The reference's own full-frame closed loop (tests/golden/frame_b8_lowrate.npz, generated from
    graphs/models/BlockBasedImgCompLossy_net.py:319-361 by tests/golden/gen_golden.py) against this
    library on the same frame and weights: symbol / index mismatches, zhat difference, PSNR and
    estimated-bpp deltas.  None when the configuration differs or the fixture is absent."""
    import numpy as np
    import torch
    path = os.path.join(ROOT, "tests", "golden", "frame_b8_lowrate.npz")
    if not os.path.exists(path) or args.config != "B8_lowrate":
        return None
    g = dict(np.load(path))
    if str(g["rate"]) != args.rate:
        return None
    import hashlib
    from lbic.layout import image_to_blocks
    H, W = int(g["H"]), int(g["W"])
    img = np.random.default_rng(int(g["image_seed"])).integers(0, 256, (1, 3, H, W), dtype=np.uint8)[0]
    if hashlib.sha256(img.tobytes()).hexdigest() != str(g["image_sha256"]):
        return dict(error="fixture frame regeneration differs")
    xb = image_to_blocks(img.astype(np.float32) / 255.0 - 0.5, arch.B)
    r = model.compress_batch(torch.from_numpy(xb)[None].to(dev), want_bits=True)
    torch.cuda.synchronize(dev)
    sym = r["symbols"][0].cpu().numpy()
    idx = r["indexes"][0].cpu().numpy()
    zh = r["zhat"][0].cpu().numpy()
    bits = r["bits"][0].cpu().numpy().astype(np.float64)
    rows = g["zhat_rows"]
    mse = float(np.mean((zh.astype(np.float64) - xb) ** 2))
    est = float(bits.sum()) / (H * W)
    est_ref = float(g["bits_per_block"].sum()) / (H * W)
    psnr, psnr_ref = -10 * np.log10(mse), float(g["psnr_db"])
    return dict(fixture="tests/golden/frame_b8_lowrate.npz: the reference's compress() closed loop on one 768x768 frame "
                        "(graphs/models/BlockBasedImgCompLossy_net.py:319-361), same weights and frame",
                symbols=int(sym.size), symbol_mismatches=int((sym != g["symbols"]).sum()),
                index_mismatches=int((idx != g["indexes"].astype(np.int32)).sum()),
                zhat_rows_max_abs_diff=float(np.abs(zh[rows] - g["zhat_row_data"]).max()),
                zhat_block_sum_max_abs_diff=float(np.abs(zh.astype(np.float64).sum(-1) - g["zhat_block_sum"]).max()),
                psnr_db=round(psnr, 6), psnr_ref_db=round(psnr_ref, 6), psnr_rel_diff=float(abs(psnr - psnr_ref) / psnr_ref),
                est_bpp=round(est, 7), est_bpp_ref=round(est_ref, 7), est_bpp_rel_diff=float(abs(est - est_ref) / est_ref))


if __name__ == "__main__":
    main()
