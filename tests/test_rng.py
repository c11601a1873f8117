"""The native restatement of torch's CPU dropout draw (gcnk_bernoulli_mt19937,
layer.host_keep_mask) against torch itself: identical keep-masks and an
identical generator state afterwards, so the stream every later draw sees is
the reference's (layer.py:185 -> ATen dropout -> bernoulli_(1 - p))."""
import numpy as np
import pytest
import torch

import gcn_amd  # noqa: F401
from graph_convolutional_networks_for_text_classification_amd import layer


@pytest.mark.parametrize("seed", [0, 7, 20260501])
@pytest.mark.parametrize("shape,p", [((7724, 200), 0.5), ((3, 5), 0.9), ((1,), 0.5), ((624,), 0.3),
                                     ((312,), 0.5), ((313,), 0.5), ((2000, 7), 0.1), ((50, 1), 1.0)])
def test_keep_mask_equals_torch_bernoulli(seed, shape, p):
    torch.manual_seed(seed)
    torch.rand(17)                       # leave the generator mid-block
    ref = torch.empty(shape, dtype=torch.float32).bernoulli_(p).to(torch.uint8)
    after_ref = torch.default_generator.get_state()
    torch.manual_seed(seed)
    torch.rand(17)
    got = layer.host_keep_mask(shape, p)
    assert layer._mt_checked
    assert torch.equal(got, ref)
    assert torch.equal(torch.default_generator.get_state(), after_ref)


def test_stream_continues_like_torch():
    """Draws interleaved with other users of the generator: masks, the values
    those users get, and the final state all match a pure-torch run."""
    def run(native):
        torch.manual_seed(3)
        out = []
        for step in range(4):
            out.append(torch.randn(5).numpy())
            if native:
                m = layer.host_keep_mask((97, 13), 0.5)
            else:
                m = torch.empty((97, 13), dtype=torch.float32).bernoulli_(0.5).to(torch.uint8)
            out.append(m.numpy())
        return out, torch.default_generator.get_state()
    a, sa = run(True)
    b, sb = run(False)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert torch.equal(sa, sb)


def test_speculative_draw_used_only_when_state_matches():
    """Back-to-back masks of one shape (the training loop) come from the
    speculative worker draw; a reseed, a changed p or shape, or another draw in
    between must discard it -- the stream stays torch's in every case."""
    def run(native):
        torch.manual_seed(11)
        out = []
        for step in range(10):
            shape, p = ((300, 40), 0.5) if step != 6 else ((300, 41), 0.5)
            if step == 3:
                torch.manual_seed(12)
            if step == 5:
                out.append(torch.rand(3).numpy())
            if step == 8:
                p = 0.8
            if native:
                m = layer.host_keep_mask(shape, p)
            else:
                m = torch.empty(shape, dtype=torch.float32).bernoulli_(p).to(torch.uint8)
            out.append(m.numpy().copy())
        return out, torch.default_generator.get_state()
    a, sa = run(True)
    b, sb = run(False)
    assert len(a) == len(b)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert torch.equal(sa, sb)


def test_native_draw_job_matches_sync_draw():
    """gcnk_bernoulli_mt19937_start/_wait (the worker-thread entry points) give
    the synchronous draw's mask and state."""
    import ctypes
    from graph_convolutional_networks_for_text_classification_amd import _lib
    lib = _lib.load()
    torch.manual_seed(5)
    b = torch.default_generator.get_state().numpy().copy()
    n = 5000
    want = np.empty(n, np.uint8)
    bs = b.copy()
    layer._mt_draw(bs, n, 0.3, want)
    left, nxt, words = layer._mt_fields(b.copy())
    st = np.ascontiguousarray(words, dtype=np.uint32)
    lf, nx = left.copy(), nxt.copy()
    got = np.empty(n, np.uint8)
    job = ctypes.c_void_p()
    assert lib.gcnk_bernoulli_mt19937_start(st.ctypes.data, lf.ctypes.data, nx.ctypes.data, n, 0.3,
                                            got.ctypes.data, ctypes.byref(job)) == 0
    assert lib.gcnk_bernoulli_mt19937_wait(job) == 0
    assert np.array_equal(got, want)
    l2, n2, w2 = layer._mt_fields(bs)
    assert np.array_equal(st, w2.astype(np.uint32)) and lf[0] == l2[0] and nx[0] == n2[0]
    assert lib.gcnk_bernoulli_mt19937_start(st.ctypes.data, lf.ctypes.data, nx.ctypes.data, n, 1.5,
                                            got.ctypes.data, ctypes.byref(job)) != 0
    assert lib.gcnk_bernoulli_mt19937_wait(None) != 0
