import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


# the experiment tests build models named after hub checkpoints (unreachable offline) on purpose with
# random-init encoder weights; test_checkpoint_host.py checks that without this opt-in it raises
os.environ.setdefault("B2P_RANDOM_W2V_WEIGHTS", "1")


def pytest_configure(config):
    # a fresh checkout carries sources only: build the HIP library (hipcc child processes, no GPU
    # touched) before anything calls torch.cuda; _lib.load() itself never builds
    from wav2vec2forbrain_amd import build_lib
    build_lib.ensure_built()
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")
    config.addinivalue_line("markers", "slow: long-running CPU oracle case")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no HIP device in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)
