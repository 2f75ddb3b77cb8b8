"""``python train.py --config configurations/craniofacial.yaml [--id ...]
[--output_path ...] [--resume] [--precision bf16]``: the reference's training
entry point (train.py) on the MI355X path (craniofacialsd-vae_amd/train.py)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import cfsd_loader  # noqa: E402

cfsd_loader.load()
from craniofacialsd_vae_amd.train import main  # noqa: E402

if __name__ == "__main__":
    main()
