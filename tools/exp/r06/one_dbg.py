"""Debug: ragged KS3311 frames through k_dec_one and the row graphs (LBIC_ONE=0) vs the encoder."""
import os, sys, types
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "learned-block-based-image-compression_amd")]
import numpy as np, torch
from lbic.arch import Arch
from lbic.model import BlockBasedImgCompLossyNetv9
from lbic.weights import synth_state_dict
arch = Arch(4, (3, 3, 1, 1), 512, 96)
cfg = types.SimpleNamespace(block_size=4, KS=[3, 3, 1, 1], N=512, M=96, gpu_device=0)
m = BlockBasedImgCompLossyNetv9(cfg)
m.load_state_dict(synth_state_dict(arch, 1337, rate="mid"))
m.update(force=True)
for Hb, Wb in [(4, 1), (2, 1), (3, 2), (3, 7), (1, 1)]:
    x = torch.from_numpy(np.random.default_rng(Hb * 100 + Wb).integers(0, 256, (1, Hb, Wb, arch.cx))
                         .astype(np.float32) / 255.0 - 0.5).cuda()
    r = m.compress_batch(x)
    st = m.entropy_encode(r["symbols"], r["indexes"])
    res = {}
    for mode in ("0", "1"):
        os.environ["LBIC_ONE"] = mode
        try:
            z = m.decompress_batch(st, Hb, Wb)
            res[mode] = (m.decode_path()["path"], bool(torch.equal(z, r["zhat"])))
        except Exception as e:
            res[mode] = str(e)[:80]
    print(Hb, Wb, res, flush=True)
