"""CLI of the reference (main.py:7-33): ``python main.py configs/<name>.json``.

Runs the reference's configs unchanged: the multi-lambda sweep (multi_agent / multi_param), the
experiments/<multi_exp_name>/exp_<lambda>/ layout, and agent dispatch by the config's "agent" name.
Under ``torchrun --nproc-per-node N`` every rank takes every N-th image (lbic.dist).
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from lbic.agent import BlockBasedImgCompLossyAgent  # noqa: E402
from lbic.config import get_config_from_json, process_config  # noqa: E402

AGENTS = {"BlockBasedImgCompLossyAgent": BlockBasedImgCompLossyAgent}   # agents/__init__.py registry


def run_agent(config):
    agent = AGENTS[config.agent](config)
    agent.run()
    agent.finalize()


def main(argv=None):
    ap = argparse.ArgumentParser(description="")
    ap.add_argument("config", metavar="config", default="None", help="The Configuration file in json format")
    args = ap.parse_args(argv)
    config, _ = get_config_from_json(args.config)
    if int(os.environ.get("WORLD_SIZE", "1")) > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get("LOCAL_RANK", "0"))
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    if config.get("multi_agent"):
        for v in config[config.multi_param]:
            config[config.multi_param] = v
            config.exp_name = os.path.join(config.multi_exp_name, "exp_" + str(v))
            run_agent(process_config(config))
    else:
        run_agent(process_config(config))


if __name__ == "__main__":
    main()
