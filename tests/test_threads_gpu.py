"""Cross-thread use of sibling handles (round 5's race class).

One thread sizes a sibling handle's workspace -- a new frame count at every call, so ensure_workspace reallocates and
zeroes its buffers and uploads its block lists -- while another thread captures (a frame count it has not coded yet)
and replays encoder graphs of the first handle on a stream of its own.  Round 5 saw two failures of this class: a
legacy-stream copy refused beside another thread's graph capture (e610271), and workspace zeroing on a non-blocking
stream overtaking the handle's previous work still queued on the caller's stream (ed23e9a).  Workspace set-up now runs
on a private stream of the handle, ordered after the caller's stream by an event (codec.hip ws_stream).  The decoding
thread runs once on a dedicated stream and once on torch's default stream (the legacy stream: what a multi-threaded
caller that never sets a stream passes).  Every call must succeed, and every result must equal the same call made
serially beforehand (encode bit for bit, decode == encode)."""
import threading
import types

import numpy as np
import pytest
import torch

from conftest import golden_arch, load_golden
from lbic.weights import synth_state_dict

pytestmark = pytest.mark.gpu


def _frames(arch, n, Hb, Wb, seed):
    rng = np.random.default_rng(seed)
    return torch.from_numpy((rng.random((n, Hb, Wb, arch.cx), dtype=np.float32) - 0.5) * 0.1).cuda()


@pytest.mark.parametrize("dec_stream", ["dedicated", "default"])
def test_workspace_resize_beside_encoder_capture(dec_stream):
    from lbic.model import BlockBasedImgCompLossyNetv9
    from lbic.streams import dedicated_streams
    g = load_golden("loop_b8_lowrate_2rows")
    arch = golden_arch(g)
    Hb, Wb = 2, 24
    cfg = types.SimpleNamespace(block_size=arch.B, KS=list(arch.KS), N=arch.N, M=arch.M, gpu_device=0)
    base = BlockBasedImgCompLossyNetv9(cfg)
    base.load_state_dict(synth_state_dict(arch, int(g["weight_seed"])))
    base.update(force=True)
    enc, dec = base.sibling(), base.sibling()
    dev = torch.device("cuda", 0)
    s_enc, s_dec = dedicated_streams(2, dev)

    # serial references: the encoder thread's frame counts 3, 5, 7, 9 (each a graph capture in the thread), the decoder
    # thread's 2, 4, 6, 8, 10 (each a workspace resize of `dec`)
    enc_n, dec_n = [3, 5, 7, 9], [2, 4, 6, 8, 10]
    xs_enc = {n: _frames(arch, n, Hb, Wb, 100 + n) for n in enc_n}
    ref_enc = {n: base.compress_batch(xs_enc[n]) for n in enc_n}
    dec_in = {}
    for n in dec_n:
        r = base.compress_batch(_frames(arch, n, Hb, Wb, 200 + n))
        dec_in[n] = (base.entropy_encode(r["symbols"], r["indexes"]), r["zhat"])
    torch.cuda.synchronize()

    errs, got_enc, got_dec = [], {}, {}
    go = threading.Barrier(2)

    def encoder():
        try:
            go.wait()
            with torch.cuda.stream(s_enc):
                for rep in range(2):                # rep 0 captures each frame count's graph, rep 1 replays it
                    for n in enc_n:
                        got_enc[(rep, n)] = enc.compress_batch(xs_enc[n])
                s_enc.synchronize()
        except BaseException as e:                  # noqa: BLE001 - surfaced below
            errs.append(e)

    def decoder():
        try:
            go.wait()
            for n in dec_n:
                if dec_stream == "dedicated":
                    with torch.cuda.stream(s_dec):
                        got_dec[n] = dec.decompress_batch(dec_in[n][0], Hb, Wb)
                        s_dec.synchronize()
                else:
                    got_dec[n] = dec.decompress_batch(dec_in[n][0], Hb, Wb)
                    torch.cuda.synchronize()
        except BaseException as e:                  # noqa: BLE001
            errs.append(e)

    ths = [threading.Thread(target=encoder), threading.Thread(target=decoder)]
    for t in ths:
        t.start()
    for t in ths:
        t.join(timeout=300)
    assert not any(t.is_alive() for t in ths), "a thread did not finish"
    assert not errs, f"{type(errs[0]).__name__}: {errs[0]}"
    torch.cuda.synchronize()
    for (rep, n), r in got_enc.items():
        for k in ("symbols", "indexes", "zhat"):
            assert torch.equal(r[k], ref_enc[n][k]), f"encode of {n} frames (pass {rep}): {k} differ"
    for n in dec_n:
        assert torch.equal(got_dec[n], dec_in[n][1]), f"decode of {n} frames != its encoder reconstruction"
