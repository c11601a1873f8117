import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    if os.environ.get("GCNK_LIB"):
        pytest.exit(f"GCNK_LIB={os.environ['GCNK_LIB']} is set: the tests check the in-tree product library only "
                    "(unset it)", returncode=4)
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


@pytest.fixture(scope="session")
def trained_golden():
    """The reference's trained model (seed 50494, trainer.py:349-376) and its
    eval logits: tests/golden/make_golden.py --trained-only."""
    import numpy as np
    import torch
    z = np.load(os.path.join(GOLDEN, "r8_trained.npz"), allow_pickle=False)
    sd = {k[3:]: torch.from_numpy(z[k].copy()) for k in z.files if k.startswith("sd_")}
    return {"state_dict": sd, "logits": z["logits"], "test_acc": float(z["test_acc"]), "epochs": int(z["epochs"]),
            "min_top2_gap": float(z["min_top2_gap"])}
