import os, sys, time
sys.path.insert(0, "learned-block-based-image-compression_amd"); sys.path.insert(0, ".")
os.environ["LBIC_DEBUG_STAMPS"] = "1"
import numpy as np, torch, types
from lbic.arch import Arch
from lbic.model import BlockBasedImgCompLossyNetv9
from lbic.weights import synth_state_dict
from lbic.layout import image_to_blocks
arch = Arch(8,(3,1,1,1),768,96)
cfg = types.SimpleNamespace(block_size=8, KS=[3,1,1,1], N=768, M=96, gpu_device=0)
m = BlockBasedImgCompLossyNetv9(cfg); m.load_state_dict(synth_state_dict(arch,1337)); m.update(force=True)
n=int(sys.argv[1]); H=int(sys.argv[2])
xb = torch.from_numpy(np.stack([image_to_blocks(np.random.default_rng(k).integers(0,256,(3,H,H)).astype(np.float32)/255-0.5,8) for k in range(n)])).cuda()
m.profile_begin(8)
for it in range(2):
    r = m.compress_batch(xb); torch.cuda.synchronize()
    st = m.entropy_encode(r["symbols"], r["indexes"])
    t0=time.perf_counter(); z = m.decompress_batch(st, H//8, H//8); torch.cuda.synchronize(); t1=time.perf_counter()
    print("decode s", t1-t0, "per step us", (t1-t0)/(H//8)**2*1e6, file=sys.stderr)
print(m.profile_end(), file=sys.stderr)
