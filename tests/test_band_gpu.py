"""Band pipeline (lbic.band, lbc_band_*): frames split into bands of block rows over ranks that hand
the two rows above each band from rank to rank, against the same frames coded whole on one GPU -- symbols, indexes
and reconstructions bit-identical.  The ranks run in torch.distributed.run children (gloo, all on cuda:0 of the
one-GPU box; tests/band_worker.py); the reference result is computed here."""
import os
import socket
import subprocess
import sys
import types

import numpy as np
import pytest
import torch

from conftest import ROOT

pytestmark = pytest.mark.gpu


def test_bands_equal_whole_frame(tmp_path):
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    import band_worker as bw
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.weights import synth_state_dict
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out = tmp_path / "bands.npz"
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=3", "--master-addr",
           "127.0.0.1", "--master-port", str(port), os.path.join(ROOT, "tests", "band_worker.py"), "--out", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    got = dict(np.load(out))
    for name, (arch, Hb, Wb, n, P, chunk) in bw.CASES.items():
        cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
        m = BlockBasedImgCompLossyNetv9(cfg)
        m.load_state_dict(synth_state_dict(arch, 1337))
        m.update(force=True)
        ref = m.compress_batch(torch.from_numpy(bw.frames(arch, Hb, Wb, n, 9)).cuda())
        for k in ("symbols", "indexes", "zhat"):
            assert np.array_equal(got[f"{name}/{k}"], ref[k].cpu().numpy()), f"{name}: {k} differ from the whole-frame encode"
