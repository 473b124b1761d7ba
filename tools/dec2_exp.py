"""Experiment: do two raster decodes of different batches overlap on one GPU (one codec handle and one HIP
stream each, a helper thread per decode; ctypes drops the GIL), and what does a concurrent encode add?
Prints alone / together wall times.  Usage: python tools/dec2_exp.py [n_img] [size] [n_dec]"""
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

n = int(sys.argv[1]) if len(sys.argv) > 1 else 32
H = int(sys.argv[2]) if len(sys.argv) > 2 else 768
ND = int(sys.argv[3]) if len(sys.argv) > 3 else 2
arch = Arch(8, (3, 1, 1, 1), 768, 96)
dev = torch.device("cuda", 0)
sd = synth_state_dict(arch, 1337)
cfg = types.SimpleNamespace(block_size=8, KS=[3, 1, 1, 1], N=768, M=96, gpu_device=0)
models = []
for _ in range(ND + 1):
    m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
    m.load_state_dict(sd)
    m.update(force=True)
    models.append(m)
Hb = Wb = H // 8
xb = torch.from_numpy(np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, H, H), dtype=np.uint8)
                                                .astype(np.float32) / 255 - 0.5, 8) for k in range(n)])).to(dev)
streams_ = [torch.cuda.Stream(dev) for _ in range(ND + 1)]


def enc(m, s):
    with torch.cuda.stream(s):
        r = m.compress_batch(xb)
        st = m.entropy_encode(r["symbols"], r["indexes"])
        torch.cuda.current_stream().synchronize()
    return st


def dec(m, s, st, out):
    with torch.cuda.stream(s):
        out.append(m.decompress_batch(st, Hb, Wb))
        torch.cuda.current_stream().synchronize()


bits = enc(models[ND], streams_[ND])
ref = []
for i in range(ND):
    dec(models[i], streams_[i], bits, ref if i == 0 else [])
torch.cuda.synchronize()
t0 = time.perf_counter(); enc(models[ND], streams_[ND]); te = time.perf_counter() - t0
t0 = time.perf_counter(); out = []; dec(models[0], streams_[0], bits, out); td = time.perf_counter() - t0
print(f"alone: encode+entropy {te*1e3:.1f} ms, decode {td*1e3:.1f} ms", flush=True)
for with_enc in (False, True):
    for rep in range(2):
        outs = [[] for _ in range(ND)]
        t0 = time.perf_counter()
        ths = [threading.Thread(target=dec, args=(models[i], streams_[i], bits, outs[i])) for i in range(ND)]
        for th in ths:
            th.start()
        te2 = 0.0
        if with_enc:
            enc(models[ND], streams_[ND])
            te2 = time.perf_counter() - t0
        for th in ths:
            th.join()
        tt = time.perf_counter() - t0
        exact = all(torch.equal(o[0], ref[0]) for o in outs)
        print(f"{ND} decodes{' + encode' if with_enc else ''}: {tt*1e3:.1f} ms (encode done at {te2*1e3:.1f}) "
              f"-> {ND * n * H * H / tt / 1e6:.2f} Mpix/s decode-side | exact {exact}", flush=True)
