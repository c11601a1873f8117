import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a ROCm GPU (MI355X); runs the HIP kernels")
    config.addinivalue_line("markers", "slow: long-running CPU test")


def pytest_collection_modifyitems(config, items):
    import torch
    if torch.cuda.is_available():
        return
    skip = pytest.mark.skip(reason="no ROCm GPU in this container")
    for it in items:
        if "gpu" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def r8():
    import gcn_amd  # noqa: F401
    from graph_convolutional_networks_for_text_classification_amd import datasets
    return datasets.load_r8_fixture(os.path.join(GOLDEN, "r8_graph.npz"))


@pytest.fixture(scope="session")
def golden_meta():
    import json
    with open(os.path.join(GOLDEN, "r8_meta.json")) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def golden_logits():
    import numpy as np
    return dict(np.load(os.path.join(GOLDEN, "r8_logits.npz"), allow_pickle=False))
