"""The drop-in boundary: module interface identical to the reference layer.py.

Checked on CPU (construction / parameters / RNG order / repr only; forward
needs the GPU)."""
import hashlib

import pytest
import torch

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import GCN, GraphConvolution


def _sha(t):
    return hashlib.sha256(t.detach().contiguous().numpy().tobytes()).hexdigest()


@pytest.mark.parametrize("seed", [50494, 99346, 0])
def test_init_reproduces_reference_parameters(r8, golden_meta, seed):
    """Same draws, same order as reference layer.py:67-82 under th.manual_seed
    (trainer.py:295): the parameter bytes hash to the reference's."""
    torch.manual_seed(seed)
    m = GCN(nfeat=r8["nfeat"], nhid=200, nclass=r8["nclass"], dropout=0.5)
    shas = golden_meta["logits"][str(seed)]["params_sha256"]
    sd = m.state_dict()
    assert list(sd) == ["gc1.weight", "gc1.bias", "gc2.weight", "gc2.bias"]
    for k, v in sd.items():
        assert _sha(v) == shas[k], k


def test_shapes_repr_and_bias_flag():
    gc = GraphConvolution(7463, 200)
    assert tuple(gc.weight.shape) == (7463, 200) and tuple(gc.bias.shape) == (200,)
    assert repr(gc) == "GraphConvolution (7463 -> 200)"
    nb = GraphConvolution(5, 3, bias=False)
    assert nb.bias is None and "bias" in dict(nb.named_parameters(recurse=False)) or nb.bias is None
    m = GCN(nfeat=100, nhid=200, nclass=20, dropout=0.5)
    assert m.dropout == 0.5
    assert sum(p.numel() for p in m.parameters()) == 100 * 200 + 200 + 200 * 20 + 20
    # trainer.py:300-303 call pattern: keyword construction
    GCN(**dict(nfeat=7, nhid=4, nclass=3, dropout=0.1))


def test_root_layer_shim_is_the_drop_in():
    import layer  # repo-root layer.py: what `from layer import GCN` (trainer.py:25) resolves to
    assert layer.GCN is GCN and layer.GraphConvolution is GraphConvolution


def test_state_dict_interchange_with_reference_layout():
    from oracle.gcn_ref import RefGCN
    torch.manual_seed(3)
    ref = RefGCN(nfeat=11, nhid=6, nclass=4, dropout=0.5)
    m = GCN(nfeat=11, nhid=6, nclass=4, dropout=0.5)
    m.load_state_dict(ref.state_dict())
    for (k1, v1), (k2, v2) in zip(ref.state_dict().items(), m.state_dict().items()):
        assert k1 == k2 and torch.equal(v1, v2)


def test_default_split_k_keeps_short_reductions_whole():
    from graph_convolutional_networks_for_text_classification_amd import ops
    assert ops.default_split_k(7724, 8, 200) == 1        # H1 W2: the skinny kernel's shape
    assert ops.default_split_k(7724, 200, 8) == 1        # g W2^T
    assert ops.default_split_k(200, 8, 7724) >= 16       # H1^T g: K = nodes


def test_release_pinned_drops_displaced_records():
    """record.release_pinned() empties the list of records kept alive for
    captured graphs (the list otherwise only grows: ADVICE round 5)."""
    from graph_convolutional_networks_for_text_classification_amd import record
    record._PINNED.append(object())
    assert record.release_pinned() >= 1
    assert record._PINNED == []
