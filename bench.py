#!/usr/bin/env python3
"""Benchmark: Mpixels/s encode+decode of the block-level masked-conv codec (BASELINE.json metric).

Workload (BASELINE.json configs[1]): B8_lowrate (B=8, KS=3,1,1,1, N=768, M=96), a batch of 32 synthetic
768x768 frames per GPU.  One step = the reference's timed region of eval_model
(agents/blkbsdimgcomp_agent.py:591-599) for the whole batch: compress (GPU wavefront closed loop + host
rANS encode, one stream per image in the reference format) and decompress (GPU raster closed loop with
GPU rANS decode).  Batches are software-pipelined: the raster decode is a chain of Hb*Wb latency-bound
steps whose cost barely grows with the rows per step, so each decoder handle decodes `gang` (default 32)
queued batches in one raster pass, and 2 such passes run side by side (own codec handle + HIP stream each),
while the next batches are compressed on the GPU (another handle/stream; `enc-gang` (default 4) batches of
distinct frames per wavefront pass) and entropy coded on host threads.
The timed region holds exactly `steps` compressions and `steps` decompressions of 32-frame batches, every
batch fully encoded and fully decoded (bit-exactness of the last one is checked).  The one-decode-in-flight
pipeline and the non-overlapped serial schedule are reported beside it ("two_stage_schedule",
"serial_schedule"; --depth 1 --gang 1 / --serial select them).
Inputs are resident in HBM when the timed region starts.  Weights are the seeded
synthetic set (lbic.weights, seed = config seed 1337); frames are seeded uint8 noise (no Kodak / no
checkpoints offline).

Multi-GPU (torchrun, one process per GPU): every rank codes its own 32 frames (weak scaling); the only
collectives are a barrier, a MAX of the step time and one all_gather of the per-image rate/distortion
summary (RCCL over xGMI).

Prints ONE JSON line on rank 0.  See DESIGN.md for the roofline definitions.
"""
import argparse
import json
import re
import math
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "learned-block-based-image-compression_amd")
for _p in (ROOT, PKG):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "Mpixels/s encode+decode, B8_lowrate N768M96, 768×768; bpp/PSNR vs ref"
PEAK_FP32_TFLOPS = 157.3     # MI355X_MICROARCH.md: f32 MFMA (dense) peak
PEAK_HBM_GBS = 8000.0        # MI355X_MICROARCH.md: HBM3E peak (spec)

CONFIGS = {   # name -> (B, KS, N, M)
    "B8_lowrate": (8, (3, 1, 1, 1), 768, 96),
    "B8_highrate": (8, (3, 3, 1, 1), 1152, 128),
    "B4_highrate": (4, (3, 3, 1, 1), 512, 96),
    "B16_lowrate": (16, (3, 1, 1, 1), 1280, 192),
}


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def cpu_baseline(arch, sd, H, W, budget_s):
    """The oracle (numpy fp32 + C rANS, one thread) on a bounded sample: the first R block rows of one
    frame, encode + decode; R chosen so the sample takes about `budget_s`."""
    from threadpoolctl import threadpool_limits
    from oracle import oracle as O
    img = np.random.default_rng(0).integers(0, 256, (3, H, W), dtype=np.uint8).astype(np.float32) / 255.0 - 0.5
    xb = O.image_to_blocks(img, arch.B)
    Hb, Wb = xb.shape[:2]
    with threadpool_limits(limits=1):
        codec = O.OracleCodec(arch, sd)

        def run(rows):
            t0 = time.perf_counter()
            out = codec.compress(xb, rows=rows)
            codec.decompress(out["bytes"], Hb, Wb, rows=rows)
            return time.perf_counter() - t0

        t1 = run(1)
        rows = int(max(1, min(Hb, math.floor(budget_s / max(t1, 1e-3)))))
        t = run(rows) if rows > 1 else t1
    px = rows * arch.B * W
    return dict(value=px / t / 1e6, unit="Mpixels/s", cores=1, kind="port",
                sample=f"oracle/oracle.py (numpy fp32, 1 thread, C rANS) encode+decode of the first {rows} of {Hb} "
                       f"block rows of one {H}x{W} frame ({rows * Wb} blocks, {t:.1f} s); per-block cost is "
                       f"content-independent, so the full frame extrapolates to {t * Hb / rows:.0f} s")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--batch", type=int, default=32, help="frames per GPU")
    ap.add_argument("--size", type=int, default=768, help="frame width (and height unless --height)")
    ap.add_argument("--height", type=int, default=0, help="frame height (default: --size)")
    ap.add_argument("--config", default="B8_lowrate", choices=sorted(CONFIGS))
    ap.add_argument("--sample-every", type=int, default=32, help="kernel-event sampling period (steps)")
    ap.add_argument("--cpu-budget", type=float, default=15.0, help="seconds of oracle CPU work (0 = skip)")
    ap.add_argument("--serial", action="store_true", help="no encode/decode overlap between consecutive batches")
    ap.add_argument("--depth", type=int, default=0,
                    help="decoder handles in flight beside the encoder (1 = two-stage pipeline; default 2).  The "
                         "raster decode is a latency-bound chain: more rows per step (--gang) and two chains side by "
                         "side fill the GPU; the process's 4 hardware queues hold the encoder, 2 decoders and the "
                         "copies.  --steps a multiple of depth x gang keeps the timed region free of a partly "
                         "filled last round of decodes")
    ap.add_argument("--gang", type=int, default=32,
                    help="batches decoded together by one decoder handle (one raster pass over gang x batch streams: "
                         "a raster step's latency barely grows with its rows)")
    ap.add_argument("--enc-gang", type=int, default=4,
                    help="batches compressed together in one wavefront pass (steps must be a multiple)")
    ap.add_argument("--enc-lds-floor", type=int, default=int(os.environ.get("LBIC_ENC_LDS_FLOOR", "0")),
                    help="LDS bytes reserved per encoder GEMM workgroup in the pipeline (>80 KB: one per CU)")
    ap.add_argument("--encode-only", type=int, default=0,
                    help="profiling aid: run this many encoder passes (enc-gang batches each) and exit (no JSON line)")
    ap.add_argument("--serial-steps", type=int, default=1, help="extra non-overlapped steps reported apart (0 = skip)")
    ap.add_argument("--substream-steps", type=int, default=2,
                    help="extra steps in the opt-in per-row sub-stream format, reported apart (0 = skip)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if dist:
        import torch.distributed as tdist
        tdist.init_process_group("nccl", device_id=dev)

    import types
    from lbic.arch import Arch
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.weights import synth_state_dict
    from lbic.layout import image_to_blocks

    B, KS, N, M = CONFIGS[args.config]
    arch = Arch(B, KS, N, M)
    W = args.size
    H = args.height or args.size
    Hb, Wb = H // B, W // B
    cfg = types.SimpleNamespace(block_size=B, KS=list(KS), N=N, M=M, gpu_device=local)
    sd = synth_state_dict(arch, 1337)

    def make_model():
        m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
        m.load_state_dict(sd)
        m.update(force=True)
        return m

    # codec handles with their own workspaces and reconstruction buffers: one encoder side and `depth`
    # decoder sides of the pipeline, each on its own HIP stream (created back to back so they land on
    # distinct hardware queues)
    depth = 0 if args.serial else (args.depth or 2)
    enc_model = make_model()
    dec_models = [make_model() for _ in range(max(depth, 1))]
    if depth and args.enc_lds_floor:
        enc_model.set_encoder_lds_floor(args.enc_lds_floor)
    s_enc = torch.cuda.Stream(dev)
    s_decs = [torch.cuda.Stream(dev) for _ in dec_models]
    handles = [enc_model] + dec_models
    plock = threading.Lock()

    n = args.batch
    # an encoder pass over `egang` batches compresses egang x n distinct frames (batch e = frames e*n .. e*n+n-1)
    egang = max(1, args.enc_gang) if depth else 1
    if args.steps % egang:
        raise SystemExit("--steps must be a multiple of --enc-gang")
    frames = np.stack([image_to_blocks(np.random.default_rng(rank * n * egang + k).integers(0, 256, (3, H, W),
                                                                                       dtype=np.uint8)
                                       .astype(np.float32) / 255.0 - 0.5, B) for k in range(n * egang)])
    xb_all = torch.from_numpy(frames).to(dev)
    xb = xb_all[:n]
    del frames

    def barrier():
        if dist:
            torch.distributed.barrier()
        torch.cuda.synchronize(dev)

    def max_over_ranks(v):
        if dist:
            t = torch.tensor([v], dtype=torch.float64, device=dev)
            torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
            v = float(t.item())
        return v

    def compress_side(ph, egang=1):
        """compress (GPU) on the encoder stream: one batch, or `egang` batches in one wavefront pass -> a list of
        per-batch results"""
        t0 = time.perf_counter()
        with torch.cuda.stream(s_enc):
            r = enc_model.compress_batch(xb if egang == 1 else xb_all)
            # symbols/indexes for the host rANS: DMA into page-locked buffers (torch's caching host allocator)
            # on the encoder's stream, ahead of the next batch's compress
            for k in ("symbols", "indexes"):
                h = torch.empty(r[k].shape, dtype=r[k].dtype, pin_memory=True)
                h.copy_(r[k], non_blocking=True)
                r[k] = h
            s_enc.synchronize()
        with plock:
            ph["encode"] += time.perf_counter() - t0
        return [dict({k: (v[e * n:(e + 1) * n] if v is not None else None) for k, v in r.items()}, frames=e)
                for e in range(egang)]

    def entropy_side(r, fmt, ph):
        """host rANS of a compressed batch (reference format: one stream per image) -> streams"""
        t0 = time.perf_counter()
        st = enc_model.entropy_encode(r["symbols"], r["indexes"], fmt=fmt, Hb=Hb, Wb=Wb)   # host tensors
        with plock:
            ph["entropy"] += time.perf_counter() - t0
        return st

    def encode_side(fmt, ph):
        r = compress_side(ph)[0]
        return r, entropy_side(r, fmt, ph)

    def decode_side(i, st, fmt, ph):
        t0 = time.perf_counter()
        with torch.cuda.stream(s_decs[i]):
            z = dec_models[i].decompress_batch(st, Hb, Wb, fmt=fmt)
            s_decs[i].synchronize()
        with plock:
            ph["decode"] += time.perf_counter() - t0
        return z

    def collect_stats():
        ks = {}
        for m_ in handles:           # merge the handles' per-kernel records
            for name, st_ in (m_.profile_end() or {}).items():
                acc = ks.setdefault(name, dict(launches=0, total_launches=0, total_ms=0.0, flops=0.0, bytes=0.0))
                for k_ in acc:
                    acc[k_] += st_[k_]
        return ks

    def run(fmt, steps, warmup, depth, label, prof=False, gang=1, egang=1):
        """`steps` timed batches.  depth 0: encode, entropy, decode one after another.  depth D >= 1: a software
        pipeline -- D decoder handles (own streams, helper threads; ctypes drops the GIL) decode `gang` batches
        per raster pass from a queue of at most D*gang encoded batches, while this thread compresses the next
        batches on the GPU and a helper thread entropy codes them on the host.  The timed region holds exactly
        `steps` encodes and `steps` decodes: the pipeline is primed with D*gang encodes and drained with D*gang
        decodes outside it (its steady state)."""
        ph = dict(encode=0.0, entropy=0.0, decode=0.0)
        scratch = dict(encode=0.0, entropy=0.0, decode=0.0)
        for i in range(warmup):
            for d in range(len(dec_models)):          # every decoder handle builds its graphs
                r, st = encode_side(fmt, scratch)
                decode_side(d, list(st) * gang, fmt, scratch)
            if egang > 1:                             # and the encoder its ganged graph
                compress_side(scratch, egang)
            log(f"[rank {rank}] {label} warmup {i + 1}/{warmup} done")
        def prof_begin():   # launch counts cover the timed region only (same sampling period: graphs are kept)
            if prof:
                for m_ in handles:
                    m_.profile_begin(args.sample_every)
        last = []
        if depth == 0:
            prof_begin()
            barrier()
            t0 = time.perf_counter()
            for i in range(steps):
                r, st = encode_side(fmt, ph)
                last = [(r, st, decode_side(0, st, fmt, ph))]
                log(f"[rank {rank}] {label} step {i + 1}/{steps}: {time.perf_counter() - t0:.2f} s")
            barrier()
            dt = max_over_ranks(time.perf_counter() - t0)
            return dt, ph, (last[-1] if last else None), collect_stats() if prof else None
        import queue
        primed = []                                 # prime (with the encoder's own pass shape: graphs are kept)
        while len(primed) < depth * gang:
            primed += [(r_, entropy_side(r_, fmt, scratch)) for r_ in compress_side(scratch, egang)]
        del primed[depth * gang:]
        prof_begin()
        q = queue.Queue(maxsize=depth * gang)      # encoded batches waiting for a decoder
        eq = queue.Queue(maxsize=1)                # compressed batches waiting for the host rANS
        done, pending = [], []
        glock = threading.Lock()

        def decoder(i):
            while True:
                items, end = [], False
                with glock:                       # one decoder gathers its whole gang
                    while len(items) < gang:      # gang decode: up to `gang` queued batches in one raster pass
                        item = q.get()
                        if item is None:
                            end = True
                            break
                        items.append(item)
                if items:
                    z_ = decode_side(i, [b for _, (_, st_) in items for b in st_], fmt, ph)
                    with plock:
                        for k, (j, (r_, st_)) in enumerate(items):
                            done.append((j, r_, st_, z_[k * n:(k + 1) * n]))
                    log(f"[rank {rank}] {label} batches {[j for j, _ in items]} decoded (decoder {i}): "
                        f"{time.perf_counter() - t0:.2f} s")
                if end:
                    q.put(None)                   # pass the end mark on to the other decoders
                    return

        def entropy_worker():
            # host rANS of batch k beside the GPU compress of batch k+1 (this thread's pool drops the GIL);
            # batches past `steps` are entropy coded inside the timed region but decoded after it (the drain)
            while True:
                item = eq.get()
                if item is None:
                    q.put(None)
                    return
                j0, rs_ = item
                for e, r_ in enumerate(rs_):
                    st_ = entropy_side(r_, fmt, ph)
                    if j0 + e < steps:
                        q.put((j0 + e, (r_, st_)))
                    else:
                        pending.append((r_, st_))

        ths = [threading.Thread(target=decoder, args=(i,)) for i in range(depth)]
        eth = threading.Thread(target=entropy_worker)
        barrier()
        t0 = time.perf_counter()
        for th in ths:
            th.start()
        for k, e in enumerate(primed[:steps]):
            q.put((k, e))
        pending.extend(primed[steps:])
        eth.start()
        for i in range(0, steps, egang):
            eq.put((len(primed) + i, compress_side(ph, egang)))
        eq.put(None)
        eth.join()
        for th in ths:
            th.join()
        barrier()
        dt = max_over_ranks(time.perf_counter() - t0)
        ks = collect_stats() if prof else None
        for k in range(0, len(pending), gang):                         # drain (outside the timed region)
            decode_side((k // gang) % depth, [b for _, st_ in pending[k:k + gang] for b in st_], fmt, scratch)
        j, r_, st_, z_ = max(done, key=lambda e: e[0])
        return dt, ph, (r_, st_, z_), ks

    # sampling is part of the captured graphs: enable it before the warmup builds them
    for m_ in handles:
        m_.profile_begin(args.sample_every)
    gang = max(1, args.gang) if depth else 1
    if args.encode_only:      # e.g. rocprofv3 --pmc on the encoder's real launch shapes (tools/gpu_profile.sh)
        for i in range(args.encode_only):
            compress_side(dict(encode=0.0, entropy=0.0, decode=0.0), egang)
            log(f"[rank {rank}] encoder pass {i + 1}/{args.encode_only} ({egang} batches) done")
        return
    run("reference", 0, args.warmup, 0, "warmup", gang=gang, egang=egang)
    dt, phase, (r, streams, z), kstats = run("reference", args.steps, 0, depth, "reference", prof=True, gang=gang,
                                             egang=egang)

    def summary(dts, phs, k):
        return dict(value=round(world * n * H * W / (dts / k) / 1e6, 4), ms_per_step=round(dts / k * 1e3, 2),
                    steps=k, phases_ms_per_step={kk: round(v / k * 1e3, 2) for kk, v in phs.items()})
    serial = two_stage = None
    if depth and args.serial_steps > 0:     # the same batches without the overlap, for reference
        dts, phs, _, _ = run("reference", args.serial_steps, 1 if gang * egang > 1 else 0, 0, "serial")
        serial = summary(dts, phs, args.serial_steps)
    if depth > 1 and args.serial_steps > 0:  # one decoder in flight
        dts, phs, _, _ = run("reference", 2 * args.serial_steps, 1 if gang * egang > 1 else 0, 1, "two-stage")
        two_stage = summary(dts, phs, 2 * args.serial_steps)

    # --- opt-in sub-stream format: same encoder, one rANS stream per block row, wavefront
    #     decode.  Reported apart from the headline (which stays on the reference bitstream format).
    sub = None
    if args.substream_steps > 0:
        run("rows", 0, 1, 0, "rows warmup")
        dts, phs, (rs, ss, zs), _ = run("rows", args.substream_steps, 0, depth, "rows")
        sub = dict(value=round(world * n * H * W / (dts / args.substream_steps) / 1e6, 4),
                   ms_per_step=round(dts / args.substream_steps * 1e3, 2), steps=args.substream_steps,
                   bpp=round(float(np.mean([len(b) * 8.0 / (H * W) for b in ss])), 5),
                   enc_dec_bit_exact_rank0=bool(torch.equal(zs, rs["zhat"])),
                   phases_ms_per_step={k: round(v / args.substream_steps * 1e3, 2) for k, v in phs.items()})

    # --- quality / consistency of the last decoded batch (outside the timed region)
    bit_exact = bool(torch.equal(z, r["zhat"]))
    xq = xb_all[r["frames"] * n:(r["frames"] + 1) * n]      # the frames of that batch
    sse = ((z - xq) ** 2).double().sum(dim=(1, 2, 3))
    rec = torch.stack([torch.tensor([float(len(s)) for s in streams], dtype=torch.float64, device=dev), sse,
                       torch.full((n,), float(H * W * 3), dtype=torch.float64, device=dev)], dim=1)
    if dist:
        allrec = [torch.empty_like(rec) for _ in range(world)]
        torch.distributed.all_gather(allrec, rec)
        rec = torch.cat(allrec)
        ok = torch.tensor([1.0 if bit_exact else 0.0], device=dev)
        torch.distributed.all_reduce(ok, op=torch.distributed.ReduceOp.MIN)
        bit_exact = bool(ok.item() == 1.0)
    rec = rec.cpu().numpy()
    bpp = float(np.mean(rec[:, 0] * 8.0 / (H * W)))
    mse = rec[:, 1] / rec[:, 2]
    psnr = float(np.mean(-10 * np.log10(mse)))

    if rank != 0:
        if dist:
            torch.distributed.destroy_process_group()
        return

    ms_step = dt / args.steps * 1e3
    px_total = world * n * H * W
    value = px_total / (dt / args.steps) / 1e6

    # --- roofline of the dominant kernel: launch spans of the sampled launches (in-kernel stamps on the
    #     GPU's 100 MHz clock, last replay of each graph in the timed region)
    roof = None
    kernels = {}
    if kstats:
        for name, s in kstats.items():
            avg = s["total_ms"] / max(s["launches"], 1)
            kernels[name] = dict(launches_sampled=s["launches"], launches_total=s["total_launches"],
                                 avg_us=round(avg * 1e3, 3),
                                 est_share_of_step=round(avg * s["total_launches"] / 1e3 / dt, 4))
        # dominant kernel: sampled average duration x true launch count over the timed region
        dom = max(kstats, key=lambda k: kstats[k]["total_ms"] / max(kstats[k]["launches"], 1) * kstats[k]["total_launches"])
        s = kstats[dom]
        t_s = s["total_ms"] / 1e3
        ai = s["flops"] / s["bytes"] if s["bytes"] else float("inf")
        ridge = PEAK_FP32_TFLOPS * 1e12 / (PEAK_HBM_GBS * 1e9)
        if s["flops"] > 0 and ai >= ridge:
            ach, peak, unit, bound = s["flops"] / t_s / 1e12, PEAK_FP32_TFLOPS, "TFLOP/s", "mfma"
        else:
            ach, peak, unit, bound = s["bytes"] / t_s / 1e9, PEAK_HBM_GBS, "GB/s", "hbm"
        traffic = None
        tfile = os.path.join(os.path.dirname(os.path.abspath(__file__)), "profiles", "pmc_traffic.json")
        if os.path.exists(tfile):       # rocprofv3 PMC passes (tools/pmc_summary.py), HBM bytes per launch
            with open(tfile) as fh:
                pm = json.load(fh)
            fam = re.sub(r"<.*>$", "", dom)
            if fam in pm and "hbm_bytes_per_dispatch" in pm[fam]:
                traffic = round(pm[fam]["hbm_bytes_per_dispatch"])
        roof = dict(kernel=dom, bound=bound, achieved=round(ach, 3), peak=peak, unit=unit,
                    frac=round(ach / peak, 5), traffic=traffic,
                    avg_launch_us=round(s["total_ms"] / s["launches"] * 1e3, 3),
                    algorithmic_per_launch=dict(flops=s["flops"] / s["launches"], bytes=s["bytes"] / s["launches"]),
                    arithmetic_intensity=round(ai, 2))
        mfma_frac = sum(v["flops"] for v in kstats.values()) / (sum(v["total_ms"] for v in kstats.values()) / 1e3) \
            / (PEAK_FP32_TFLOPS * 1e12)
        roof["all_kernels_mfma_frac"] = round(mfma_frac, 5)
    # whole-step algorithmic work
    mac_enc, mac_dec = arch.live_macs_per_block()
    step_flops = 2.0 * (mac_enc + mac_dec) * Hb * Wb * n
    cpu = None
    if args.cpu_budget > 0 and world == 1:
        cpu = cpu_baseline(arch, sd, H, W, args.cpu_budget)

    out = {
        "metric": METRIC, "value": round(value, 4), "unit": "Mpixels/s", "n_gpus": world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": round(ms_step, 2), "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "f32",
        "data": "synthetic: seeded uint8 noise frames, seeded synthetic weights (no checkpoints / Kodak offline)",
        "config": {"workload": f"{args.config} N{N}M{M}, batch of {n} synthetic {H}x{W} frames per GPU, "
                               "encode+decode in the reference bitstream format (one raster rANS stream per image)",
                   "batch_per_gpu": n, "frame": [H, W], "parallelism": f"images sharded over {world} GPU(s)",
                   "global_batch": n * world,
                   "schedule": "serial: encode, entropy, decode per batch" if depth == 0 else
                   f"software pipeline: {depth} raster decode pass(es) in flight (one codec handle + HIP stream "
                   f"each), each over {gang} queued batches, beside the GPU compress and host rANS of the next "
                   f"batches (own handle + stream, host threads); each timed step = one full encode and one full "
                   f"decode of a {n}-frame batch",
                   "decode_passes_in_flight": depth, "batches_per_decode_pass": gang,
                   "batches_per_encode_pass": egang},
        "roofline": roof, "cpu_baseline": cpu,
        "quality": {"bpp": round(bpp, 5), "psnr_db": round(psnr, 3), "enc_dec_bit_exact": bit_exact},
        "phases_ms_per_step": {k: round(v / args.steps * 1e3, 2) for k, v in phase.items()},
        "step_algorithmic_tflop": round(step_flops / 1e12, 3),
        "step_mfma_frac": round(step_flops / (dt / args.steps) / (PEAK_FP32_TFLOPS * 1e12), 5),
        "kernels": kernels,
        "serial_schedule": serial,
        "two_stage_schedule": two_stage,
        "substream_format": sub,
    }
    print(json.dumps(out), flush=True)
    if dist:
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
