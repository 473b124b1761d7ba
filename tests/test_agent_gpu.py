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
