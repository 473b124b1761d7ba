"""Experiment: how many 32-frame raster decodes overlap on one GPU?  ND decodes of the same batch side by side
(one codec handle, one HIP stream and one host thread each), no encoder, for ND = 1..4, with the streams made by
torch's stream pool (`pool`) or created raw through hipStreamCreateWithFlags (`raw`, so the hardware-queue
assignment follows this script's creation order).  Prints wall time per configuration.
Usage: python tools/decN_exp.py [pool|raw] [size] [max_nd]"""
import ctypes
import os
import sys
import threading
import time
import types

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "learned-block-based-image-compression_amd"))
from lbic.arch import Arch  # noqa: E402
from lbic.layout import image_to_blocks  # noqa: E402
from lbic.model import BlockBasedImgCompLossyNetv9  # noqa: E402
from lbic.weights import synth_state_dict  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "pool"
H = int(sys.argv[2]) if len(sys.argv) > 2 else 384
MAXND = int(sys.argv[3]) if len(sys.argv) > 3 else 4
n = 32
arch = Arch(8, (3, 1, 1, 1), 768, 96)
dev = torch.device("cuda", 0)
sd = synth_state_dict(arch, 1337, rate="low")
cfg = types.SimpleNamespace(block_size=8, KS=[3, 1, 1, 1], N=768, M=96, gpu_device=0)


def make():
    m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
    m.load_state_dict(sd)
    m.update(force=True)
    return m


if mode == "raw":
    hip = ctypes.CDLL("libamdhip64.so")
    raw = []
    for _ in range(MAXND + 1):
        s = ctypes.c_void_p()
        assert hip.hipStreamCreateWithFlags(ctypes.byref(s), ctypes.c_uint(1)) == 0
        raw.append(s.value)
    streams = [torch.cuda.ExternalStream(p, device=dev) for p in raw]
else:
    streams = [torch.cuda.Stream(dev) for _ in range(MAXND + 1)]
models = [make() for _ in range(MAXND + 1)]
Hb = Wb = H // 8
xb = torch.from_numpy(np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, H, H), dtype=np.uint8)
                                                .astype(np.float32) / 255 - 0.5, 8) for k in range(n)])).to(dev)
with torch.cuda.stream(streams[MAXND]):
    r = models[MAXND].compress_batch(xb)
    torch.cuda.current_stream().synchronize()
bits = models[MAXND].entropy_encode(r["symbols"], r["indexes"])


def dec(i, out):
    with torch.cuda.stream(streams[i]):
        out.append(models[i].decompress_batch(bits, Hb, Wb))
        torch.cuda.current_stream().synchronize()


for i in range(MAXND):      # graphs built, workspaces allocated
    dec(i, [])
torch.cuda.synchronize()
print(f"mode {mode}, {n} x {H}x{H}, GPU_MAX_HW_QUEUES={os.environ.get('GPU_MAX_HW_QUEUES', 'default')}", flush=True)
t1 = None
for nd in range(1, MAXND + 1):
    for rep in range(2):
        outs = [[] for _ in range(nd)]
        t0 = time.perf_counter()
        ths = [threading.Thread(target=dec, args=(i, outs[i])) for i in range(nd)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        tt = time.perf_counter() - t0
        if nd == 1 and rep == 1:
            t1 = tt
        exact = all(torch.equal(o[0], r["zhat"]) for o in outs)
        print(f"  {nd} decodes: {tt * 1e3:8.1f} ms  ({nd * n * H * H / tt / 1e6:6.2f} Mpix/s decode-side"
              f"{'' if t1 is None else f', {nd * t1 / tt:.2f}x of serial'}) exact {exact}", flush=True)
