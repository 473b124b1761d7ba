"""``BlockBasedImgCompLossyAgent`` -- the reference's agent for the hot path (mode ``eval_model``).

Mirrors agents/blkbsdimgcomp_agent.py:22-104 (construction, checkpoint) and :552-641 (update_model,
eval_model), agents/base.py:89-128 (load_checkpoint), :165-207 (run), :238-240 (finalize), on the HIP
codec.  Per image it does what eval_model does: shift to [-1/2, 1/2], replicate-pad to a multiple of B,
block->channel layout, timed compress / decompress, encoder/decoder agreement, bpp / MSE / PSNR /
MS-SSIM, reconstruction PNG, and the same log lines.  Training modes are out of scope and
raise.  Under torchrun the images are sharded over the ranks and the summary is all-gathered.
"""
from __future__ import annotations

import glob
import logging
import math
import os
import time

import numpy as np
import torch
import torch.nn.functional as F

from . import dist as D
from .layout import arrange_block_pixels_to_channel_dim, arrange_channel_dim_to_block_pixels
from .metrics import ms_ssim
from .model import BlockBasedImgCompLossyNetv9
from .weights import load_reference_checkpoint, rate_for_lambda, synth_state_dict

IMG_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".ppm")


class RDMeter:
    """loggers/rate.py RDLogger: running means and the 'Valid Epoch' line (:119-138)."""

    def __init__(self):
        self.rows = []
        self.logger = logging.getLogger("Loss")

    def __call__(self, loss, mse, rate):
        self.rows.append((loss, mse, rate))

    def display(self, typ="va", epoch=0):
        a = np.asarray(self.rows, np.float64)
        loss, mse, rate = (a.mean(0) if len(a) else (0.0, 1.0, 0.0))
        psnr = 10 * math.log10(1.0 / mse)
        now = time.strftime("%H:%M:%S")
        self.logger.info("  Valid Epoch: {:3d}  RDLoss: {:.6f} {}: {:.6f}/{:.2f} Rate: {:.3f} ({})".format(
            epoch, loss, "MSE/PSNR", mse, psnr, rate, now))
        return loss, mse, rate, 0.0


def _list_images(folder):
    if not folder or not os.path.isdir(folder):
        raise FileNotFoundError(f"valid_data folder not found: {folder!r} (config key valid_data)")
    files = sorted(f for f in glob.glob(os.path.join(folder, "*")) if f.lower().endswith(IMG_EXT))
    if not files:
        raise FileNotFoundError(f"no images in {folder}")
    return files


def _load_image(path):
    from PIL import Image
    with open(path, "rb") as f:
        img = Image.open(f).convert("RGB")
        a = np.asarray(img, dtype=np.uint8).copy()
    return torch.from_numpy(a).permute(2, 0, 1).float().div(255.0)[None]      # [1, 3, H, W] in [0, 1]


def _save_image(x01, path):
    from PIL import Image
    a = (x01.clamp(0, 1).mul(255).add(0.5).floor()).byte().permute(1, 2, 0).cpu().numpy()
    Image.fromarray(a).save(path)


class BlockBasedImgCompLossyAgent:
    def __init__(self, config):
        self.config = config
        self.logger = logging.getLogger("Agent")
        if getattr(config, "net_version", "v9") != "v9":
            raise NotImplementedError("only net_version v9 (every reference config) is implemented")
        if not (getattr(config, "cuda", True) and torch.cuda.is_available()):
            raise RuntimeError("the codec runs on the GPU (HIP kernels); no GPU is visible")
        self.rank, self.world = D.rank_world()
        local = int(os.environ.get("LOCAL_RANK", getattr(config, "gpu_device", 0) or 0))
        self.device = torch.device("cuda", local)
        torch.cuda.set_device(self.device)
        self.block_size = int(config.block_size)
        self.model0 = BlockBasedImgCompLossyNetv9(config, device=self.device)
        self.lambda_ = config.lambda_
        self.rcrec_logger = RDMeter()
        if config.mode in ("eval_model", "update_model", "validate_recu_reco_fast"):
            self.load_checkpoint(config.modelbest_file_load)

    # agents/base.py:89-128 (eval checkpoints: {'state_dict0': sd}); a missing file is loud here
    def load_checkpoint(self, filename):
        path = os.path.join(getattr(self.config, "checkpoint_dir", ""), filename)
        if os.path.exists(path):
            self.logger.info("Loading checkpoint '{}'".format(path))
            self.model0.load_state_dict(load_reference_checkpoint(path), strict=True)
        else:
            lam = self.lambda_[0] if isinstance(self.lambda_, (list, tuple)) else self.lambda_
            rate = rate_for_lambda(lam)
            self.logger.warning("!!! No checkpoint exists at '{}'. Continuing with SYNTHETIC seeded weights "
                                "(seed {}, '{}' operating point for lambda {}) -- rate/PSNR are not those of a trained "
                                "model.".format(path, self.config.seed, rate, lam))
            self.model0.load_state_dict(synth_state_dict(self.model0.arch, int(self.config.seed), rate=rate))

    def run(self):
        mode = self.config.mode
        if mode == "eval_model":
            return self.eval_model()
        if mode == "update_model":
            return self.update_model(force=True)
        if mode == "validate_recu_reco_fast":
            return self.validate_recu_reco_fast()
        if mode in ("test", "validate", "validate_recu_reco", "gen_train_set",
                    "gen_train_set_postproc", "train_postproc_mdl", "train_one_acl", "train_all_acl", "debug",
                    "model_size_estimation", "flops_estimation"):
            raise NotImplementedError(f"mode {mode!r} is outside the accelerated hot path (SURVEY §2)")
        raise NameError("'" + mode + "'" + " is not a valid training mode.")

    def update_model(self, force=False):
        """agents/blkbsdimgcomp_agent.py:552-558 (also writes '<file>_updated')."""
        self.model0.update(force=force)
        if self.rank == 0 and getattr(self.config, "checkpoint_dir", None):
            fname = os.path.join(self.config.checkpoint_dir, self.config.modelbest_file_load + "_updated")
            torch.save({"state_dict0": self.model0.state_dict()}, fname)

    @torch.no_grad()
    def eval_model(self):
        """agents/blkbsdimgcomp_agent.py:561-641."""
        self.update_model(force=True)
        L = self.model0.arch.lru
        B = self.block_size
        files = _list_images(self.config.valid_data)
        mine = D.shard(list(enumerate(files)), self.rank, self.world)
        recs = []
        out_dir = os.path.join(self.config.checkpoint_dir, "..", os.path.basename(os.path.normpath(self.config.valid_data)))
        os.makedirs(out_dir, exist_ok=True)
        for batch_idx, path in mine:
            x = _load_image(path).to(self.device) - 0.5
            h, w = x.size(2), x.size(3)
            nh, nw = (h + B - 1) // B * B, (w + B - 1) // B * B
            pb, pr = nh - h, nw - w
            xp = F.pad(x, (0, pr, 0, pb), mode="replicate")
            xp = arrange_block_pixels_to_channel_dim(xp, B)
            torch.cuda.synchronize(self.device)
            t0 = time.time()
            bitstream, xhat_enc = self.model0.compress(xp, [L, L, L], self.config.M)
            torch.cuda.synchronize(self.device)
            enc_time = time.time() - t0
            t0 = time.time()
            xhat_dec = self.model0.decompress(bitstream, [L, L, L], xp.shape, self.config.M, xp.device)
            torch.cuda.synchronize(self.device)
            dec_time = time.time() - t0
            dif = torch.abs(xhat_enc - xhat_dec)
            img_enc = arrange_channel_dim_to_block_pixels(xhat_enc, B)[:, :, :h, :w]
            num_pixels = x.size(0) * h * w
            bpp = len(bitstream) * 8.0 / num_pixels
            mse = F.mse_loss(x, img_enc).item()
            rd_loss = bpp + self.lambda_ * mse
            psnr = -10 * math.log10(mse)
            msssim = ms_ssim(x + 0.5, img_enc + 0.5, data_range=1.0).item()
            msssimdb = -10 * math.log10(max(1.0 - msssim, 1e-12)) if msssim == msssim else float("nan")
            name = os.path.basename(path)
            _save_image(img_enc[0] + 0.5, os.path.join(out_dir, name))
            self.logger.info("Image {:2d} --> ".format(batch_idx) + (
                "RDLoss:{:.3f} MSE/PSNR:{:.5f}/{:.2f} Rate:{:.3f} MS-SSIM/dB:{:.6f}/{:.2f} Enc/DecTime:{:.1f}/{:.1f} "
                "Enc-Dec.Mad/Max/Min:{:.2f}/{:.2f}/{:.2f} ({})").format(
                rd_loss, mse, psnr, bpp, msssim, msssimdb, enc_time, dec_time, dif.mean().item() * 255,
                dif.max().item() * 255, dif.min().item() * 255, name))
            recs.append([batch_idx, rd_loss, mse, bpp, msssim, msssimdb, enc_time, dec_time])
        rec = torch.tensor(recs, dtype=torch.float64, device=self.device).reshape(-1, 8)
        allrec = D.gather_records(rec).cpu().numpy()
        allrec = allrec[np.argsort(allrec[:, 0])]
        if self.rank == 0:
            for r in allrec:
                self.rcrec_logger(r[1], r[2], r[3])
            self.rcrec_logger.display(typ="va")
            self.logger.info(f"avg_psnr = {np.mean(-10 * np.log10(allrec[:, 2])):.2f}  "
                             f"avg_msssim = {np.mean(allrec[:, 4]):.8f} avg_msssimdb = {np.mean(allrec[:, 5]):.2f}")
        return allrec

    @torch.no_grad()
    def validate_recu_reco_fast(self):
        """agents/blkbsdimgcomp_agent.py:491-528: recursive (closed-loop) reconstruction of each validation
        image with the estimated rate of forward(), no entropy coding.  The reference's valid loader
        center-crops to val_patch_size (dataloaders/image_dl_ACL.py:119); the crop is rounded down to whole
        blocks here.  Loss as TrainRDLoss.forward (graphs/losses/rate_dist.py:41-50): rate + lambda * mse,
        rate = sum(self-information) / numel(x) * 3."""
        B = self.block_size
        files = _list_images(self.config.valid_data)
        mine = D.shard(list(enumerate(files)), self.rank, self.world)
        out_dir = os.path.join(self.config.checkpoint_dir, "..", "valid_set")
        os.makedirs(out_dir, exist_ok=True)
        recs = []
        for batch_idx, path in mine:
            x = _load_image(path).to(self.device)
            h, w = x.size(2), x.size(3)
            ps = getattr(self.config, "val_patch_size", None)
            if ps:
                ch, cw = (ps, ps) if isinstance(ps, int) else (int(ps[0]), int(ps[1]))
                ch, cw = min(ch, h), min(cw, w)
                t, l = int(round((h - ch) / 2.0)), int(round((w - cw) / 2.0))   # torchvision CenterCrop
                x = x[:, :, t:t + ch, l:l + cw]
                h, w = ch, cw
            h, w = h // B * B, w // B * B
            x = arrange_block_pixels_to_channel_dim(x[:, :, :h, :w] - 0.5, B)
            zhat, info = self.model0.validate_recu_reco(x)
            mse = F.mse_loss(x, zhat).item()
            rate = (info.sum() / x.numel() * 3).item()
            rd_loss = rate + self.lambda_ * mse
            psnr = 10.0 * math.log10(1.0 / mse)
            self.logger.info("Image {:2d} --> ".format(batch_idx) +
                             "RDLoss:{:.3f} MSE/PSNR:{:.5f}/{:.2f} Rate:{:.3f}".format(rd_loss, mse, psnr, rate))
            img = arrange_channel_dim_to_block_pixels(zhat + 0.5, B)
            _save_image(img[0], os.path.join(out_dir, "valid_reco_{:d}.png".format(batch_idx)))
            recs.append([batch_idx, rd_loss, mse, rate])
        rec = torch.tensor(recs, dtype=torch.float64, device=self.device).reshape(-1, 4)
        allrec = D.gather_records(rec).cpu().numpy()
        allrec = allrec[np.argsort(allrec[:, 0])]
        if self.rank == 0:
            for r in allrec:
                self.rcrec_logger(r[1], r[2], r[3])
            loss = self.rcrec_logger.display(typ="va")
            self.logger.info(f"avg_psnr = {np.mean(-10 * np.log10(allrec[:, 2])):.2f}")
            return loss
        return None

    def finalize(self):
        self.logger.info("Please wait while finalizing the operation.. Thank you")
