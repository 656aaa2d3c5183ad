"""CPU checks of the BN-backward fusion hand-off (ops/bnfuse.py): matches only the exact
(z, y) pair, misses fall back, dead tensors never match."""
import gc

import torch

from featurenet_amd.ops import bnfuse


def test_source_and_take_match_only_the_tagged_pair(monkeypatch):
    monkeypatch.setenv("FN_BN_DGRAD_FUSE", "1")
    y = torch.randn(2, 4, 4, 4, 8)
    prm = torch.randn(4, 8)
    z = torch.relu(y)
    bnfuse.tag_output(z, y, prm, 1)
    src = bnfuse.source_of(z.reshape(2, 4, 4, 4, 8))      # a same-extent view matches
    assert src is not None and src[0] is y and src[1] is prm and src[2] == 1
    assert bnfuse.source_of(torch.empty_like(z)) is None  # another tensor does not
    dz = torch.randn_like(z)
    slab = torch.randn(3, 2, 8)
    bnfuse.offer(dz, slab, y)
    assert bnfuse.take(dz, torch.empty_like(y)) is None   # wrong y: no slab (and the entry is consumed)
    bnfuse.offer(dz, slab, y)
    assert bnfuse.take(dz, y) is slab
    assert bnfuse.take(dz, y) is None                     # taken once


def test_dead_outputs_do_not_match(monkeypatch):
    monkeypatch.setenv("FN_BN_DGRAD_FUSE", "1")
    y = torch.randn(64)
    prm = torch.randn(4, 1)
    z = torch.relu(y)
    ptr = z.data_ptr()
    bnfuse.tag_output(z, y, prm, 1)
    del z
    gc.collect()
    w = torch.empty(64)
    if w.data_ptr() == ptr:                               # allocator reuse must not resurrect the entry
        assert bnfuse.source_of(w) is None
    monkeypatch.setenv("FN_BN_DGRAD_FUSE", "0")
    z2 = torch.relu(y)
    bnfuse.tag_output(z2, y, prm, 1)
    assert bnfuse.source_of(z2) is None                   # disabled: nothing is recorded
