"""JSON config handling with the reference's semantics (utils/config.py:50-116), without easydict."""
from __future__ import annotations

import json
import logging
import os
from logging import Formatter
from logging.handlers import RotatingFileHandler


class AttrDict(dict):
    """dict with attribute access (what the reference gets from EasyDict)."""

    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError as e:
            raise AttributeError(k) from e

    def __setattr__(self, k, v):
        self[k] = v


def get_config_from_json(json_file):
    """utils/config.py:50-66."""
    with open(json_file) as f:
        d = json.load(f)
    return AttrDict(d), d


_LOGGING_SET = False


def setup_logging(log_dir):
    """utils/config.py:25-47: console + rotating exp_debug.log / exp_error.log."""
    global _LOGGING_SET
    if _LOGGING_SET:
        return
    fmt_file = "[%(levelname)s] - %(asctime)s - %(name)s - : %(message)s in %(pathname)s:%(lineno)d"
    root = logging.getLogger()
    root.setLevel(logging.INFO)
    ch = logging.StreamHandler()
    ch.setLevel(logging.INFO)
    ch.setFormatter(Formatter("[%(levelname)s]: %(message)s"))
    fh = RotatingFileHandler(os.path.join(log_dir, "exp_debug.log"), maxBytes=10 ** 6, backupCount=5)
    fh.setLevel(logging.DEBUG)
    fh.setFormatter(Formatter(fmt_file))
    eh = RotatingFileHandler(os.path.join(log_dir, "exp_error.log"), maxBytes=10 ** 6, backupCount=5)
    eh.setLevel(logging.WARNING)
    eh.setFormatter(Formatter(fmt_file))
    for h in (ch, fh, eh):
        root.addHandler(h)
    _LOGGING_SET = True


def process_config(config, root="experiments"):
    """utils/config.py:69-102: experiments/<exp_name>/{summaries,checkpoints,out,logs}/ + logging."""
    if "exp_name" not in config:
        raise ValueError("Please provide the exp_name in json file")
    config.summary_dir = os.path.join(root, config.exp_name, "summaries/")
    config.checkpoint_dir = os.path.join(root, config.exp_name, "checkpoints/")
    config.out_dir = os.path.join(root, config.exp_name, "out/")
    config.log_dir = os.path.join(root, config.exp_name, "logs/")
    for d in (config.summary_dir, config.checkpoint_dir, config.out_dir, config.log_dir):
        os.makedirs(d, exist_ok=True)
    setup_logging(config.log_dir)
    logging.getLogger().info("The pipeline of the project will begin now.")
    return config
