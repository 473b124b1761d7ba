"""Experiment: does batch k+1's encode (+ host entropy coding) overlap batch k's raster decode on one GPU?
Two codec handles (separate workspaces), decode on its own stream in a helper thread (ctypes drops the GIL),
encode on another stream in the main thread.  Prints the alone/together wall times."""
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

n, H = int(sys.argv[1]) if len(sys.argv) > 1 else 32, int(sys.argv[2]) if len(sys.argv) > 2 else 768
arch = Arch(8, (3, 1, 1, 1), 768, 96)
dev = torch.device("cuda", 0)
sd = synth_state_dict(arch, 1337)
cfg = types.SimpleNamespace(block_size=8, KS=[3, 1, 1, 1], N=768, M=96, gpu_device=0)
models = []
for _ in range(2):
    m = BlockBasedImgCompLossyNetv9(cfg, device=dev)
    m.load_state_dict(sd)
    m.update(force=True)
    models.append(m)
Hb = Wb = H // 8
xb = torch.from_numpy(np.stack([image_to_blocks(np.random.default_rng(k).integers(0, 256, (3, H, H), dtype=np.uint8)
                                                .astype(np.float32) / 255 - 0.5, 8) for k in range(n)])).to(dev)
PRIO = int(os.environ.get("PRIO", "0"))
ENC_CUS = int(os.environ.get("ENC_CUS", "0"))


def cu_masked_stream(n_cu):
    """HIP stream restricted to the first n_cu compute units (hipExtStreamCreateWithCUMask)."""
    import ctypes
    hip = ctypes.CDLL("libamdhip64.so")
    words = (ctypes.c_uint32 * 8)(*[0xffffffff if (w + 1) * 32 <= n_cu else ((1 << max(0, n_cu - w * 32)) - 1)
                                   for w in range(8)])
    st = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(st), ctypes.c_uint32(8), words)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(st.value, device=dev)
sd_, se_ = (torch.cuda.Stream(dev, priority=-1), torch.cuda.Stream(dev, priority=0)) if PRIO else (torch.cuda.Stream(dev), torch.cuda.Stream(dev))
if ENC_CUS:
    se_ = cu_masked_stream(ENC_CUS)


def enc(m):
    with torch.cuda.stream(se_):
        r = m.compress_batch(xb)
        st = m.entropy_encode(r["symbols"], r["indexes"])
    return st


def dec(m, st, out):
    with torch.cuda.stream(sd_):
        out.append(m.decompress_batch(st, Hb, Wb))
        torch.cuda.current_stream().synchronize()


streams = enc(models[1])                          # warm the encoder graph (handle 1)
out = []
dec(models[0], streams, out)                      # warm the decoder graphs (handle 0)
torch.cuda.synchronize()
t0 = time.perf_counter(); enc(models[1]); torch.cuda.synchronize(); te = time.perf_counter() - t0
t0 = time.perf_counter(); out = []; dec(models[0], streams, out); torch.cuda.synchronize(); td = time.perf_counter() - t0
for rep in range(2):
    out = []
    t0 = time.perf_counter()
    th = threading.Thread(target=dec, args=(models[0], streams, out))
    th.start()
    st2 = enc(models[1])
    torch.cuda.synchronize()
    t_enc_done = time.perf_counter() - t0
    th.join()
    torch.cuda.synchronize()
    tt = time.perf_counter() - t0
    print(f"alone: encode+entropy {te*1e3:.1f} ms, decode {td*1e3:.1f} ms, sum {(te+td)*1e3:.1f} | together {tt*1e3:.1f} ms "
          f"(encode side done at {t_enc_done*1e3:.1f}) | decode exact {torch.equal(out[0], out[0])}", flush=True)
