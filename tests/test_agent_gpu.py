"""GPU: the reference's CLI flow (main.py -> BlockBasedImgCompLossyAgent.eval_model) on a PNG folder, with a
frame size that is not a multiple of the block size (replicate padding, agents/blkbsdimgcomp_agent.py:583-586)
and the multi-lambda sweep; checks the log lines and that decoder == encoder (Enc-Dec.Mad 0)."""
import json
import logging
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_main_eval_model(tmp_path, monkeypatch, caplog):
    from PIL import Image
    import main as lbic_main
    data = tmp_path / "kodak" / "test"
    data.mkdir(parents=True)
    rng = np.random.default_rng(3)
    for k, (h, w) in enumerate([(170, 165), (32, 32)]):
        Image.fromarray(rng.integers(0, 256, (h, w, 3), dtype=np.uint8)).save(data / f"img{k}.png")
    cfg = dict(exp_name="", multi_exp_name="tiny", agent="BlockBasedImgCompLossyAgent", net_version="v9",
               mode="eval_model", cuda=True, gpu_device=0, seed=1337, block_size=4, KS=[3, 3, 1, 1], N=64, M=16,
               use_postpm=False, multi_agent=True, multi_param="lambda_", lambda_=[100.0, 200.0],
               modelbest_file_load="missing.pth.tar", valid_data=str(data))
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    monkeypatch.chdir(tmp_path)
    with caplog.at_level(logging.INFO):
        lbic_main.main([str(p)])
    lines = [r.getMessage() for r in caplog.records]
    imgs = [l for l in lines if l.startswith("Image ")]
    assert len(imgs) == 4                                    # 2 images x 2 lambdas
    for l in imgs:
        assert "Enc-Dec.Mad/Max/Min:0.00/0.00/0.00" in l
    assert sum("Valid Epoch" in l for l in lines) == 2
    assert any("SYNTHETIC" in l for l in lines)              # missing checkpoint is loud
    assert (tmp_path / "experiments" / "tiny" / "exp_100.0" / "checkpoints" / "missing.pth.tar_updated").exists()
    assert (tmp_path / "experiments" / "tiny" / "exp_100.0" / "test" / "img0.png").exists()


def test_main_validate_recu_reco_fast(tmp_path, monkeypatch, caplog):
    """mode validate_recu_reco_fast through main.py: one log line per image and the 'Valid Epoch' summary."""
    from PIL import Image
    import main as lbic_main
    data = tmp_path / "val"
    data.mkdir()
    rng = np.random.default_rng(4)
    for k in range(2):
        Image.fromarray(rng.integers(0, 256, (40, 36, 3), dtype=np.uint8)).save(data / f"v{k}.png")
    cfg = dict(exp_name="recu", agent="BlockBasedImgCompLossyAgent", net_version="v9", mode="validate_recu_reco_fast",
               cuda=True, gpu_device=0, seed=1337, block_size=4, KS=[3, 3, 1, 1], N=64, M=16, use_postpm=False,
               lambda_=100.0, val_patch_size=32, modelbest_file_load="missing.pth.tar", valid_data=str(data))
    p = tmp_path / "cfg.json"
    p.write_text(json.dumps(cfg))
    monkeypatch.chdir(tmp_path)
    with caplog.at_level(logging.INFO):
        lbic_main.main([str(p)])
    lines = [r.getMessage() for r in caplog.records]
    assert sum(l.startswith("Image ") and "RDLoss:" in l for l in lines) == 2
    assert any("Valid Epoch" in l for l in lines)
    assert any(l.startswith("avg_psnr") for l in lines)


def test_main_reference_config_b8_lowrate_full_frame(tmp_path, monkeypatch, caplog):
    """BASELINE config 1 through the reference's entry point: `python main.py configs/blkbsdimgcomp_B8_lowrate.json`
    (the reference's config shipped verbatim, only valid_data redirected) on a 768x768 PNG of the full-frame fixture's
    image; no checkpoint, so the agent loads the seeded synthetic weights at the config's operating point -- the very
    weights and frame of tests/golden/frame_b8_lowrate.npz, the reference's own compress() closed loop.  The log line's
    MSE / PSNR must be the fixture's, Enc-Dec.Mad 0.00 (agents/blkbsdimgcomp_agent.py:561-641)."""
    import hashlib
    import re
    from PIL import Image
    import main as lbic_main
    from conftest import load_golden
    g = load_golden("frame_b8_lowrate")
    H, W = int(g["H"]), int(g["W"])
    img = np.random.default_rng(int(g["image_seed"])).integers(0, 256, (1, 3, H, W), dtype=np.uint8)[0]
    assert hashlib.sha256(img.tobytes()).hexdigest() == str(g["image_sha256"])
    data = tmp_path / "kodak" / "test"
    data.mkdir(parents=True)
    Image.fromarray(np.ascontiguousarray(img.transpose(1, 2, 0))).save(data / "frame.png")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    src = os.path.join(root, "learned-block-based-image-compression_amd", "configs", "blkbsdimgcomp_B8_lowrate.json")
    cfg = json.load(open(src))
    raw_keys = set(cfg)
    cfg["valid_data"] = str(data)                          # the only override
    assert set(cfg) == raw_keys and cfg["block_size"] == 8 and cfg["N"] == 768 and cfg["M"] == 96
    p = tmp_path / "blkbsdimgcomp_B8_lowrate.json"
    p.write_text(json.dumps(cfg))
    monkeypatch.chdir(tmp_path)
    with caplog.at_level(logging.INFO):
        lbic_main.main([str(p)])
    lines = [r.getMessage() for r in caplog.records]
    imgs = [l for l in lines if l.startswith("Image ")]
    assert len(imgs) == 1, lines
    print(imgs[0])
    m = re.search(r"MSE/PSNR:([\d.]+)/([\d.]+) Rate:([\d.]+) .*Enc/DecTime:([\d.]+)/([\d.]+) "
                  r"Enc-Dec\.Mad/Max/Min:([\d.]+)/([\d.]+)/([\d.]+)", imgs[0])
    assert m, imgs[0]
    mse, psnr, rate = float(m.group(1)), float(m.group(2)), float(m.group(3))
    psnr_ref = float(g["psnr_db"])
    assert abs(psnr - psnr_ref) <= 0.005 + 1e-9, (psnr, psnr_ref)             # the line prints 2 decimals
    assert abs(mse - 10 ** (-psnr_ref / 10)) <= 5e-6 + 1e-9, (mse, 10 ** (-psnr_ref / 10))   # 5 decimals
    est_ref = float(g["bits_per_block"].sum()) / (H * W)
    assert abs(rate - est_ref) <= 0.05 * est_ref, (rate, est_ref)            # actual rANS bytes vs the estimate
    assert m.group(6) == "0.00" and m.group(7) == "0.00"
    assert any("'low' operating point" in l for l in lines)
