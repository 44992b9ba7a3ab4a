"""Host logic of kernels._LadderRing (the gradient path's deferred ladder
outcome for qEHVI / qNEHVI) with stand-in pinned blocks and events: a
backward settles its own forward only, a block that comes round again
reports the forward that left it pending (one ring behind), the poll reports
the pending ones oldest first, and outcomes raise / warn as the per-member
psd_safe_cholesky checks would."""
import warnings

import pytest

from botorch_amd import kernels
from botorch_amd.exceptions import NotPSDError, NumericalWarning


class _Block:
    def __init__(self):
        self.words = [0.0] * 16

    def arm(self, m):
        for i in range(2 * m):
            self.words[i] = 0.0
        return [(i, i) for i in range(m)]


class _Event:
    def __init__(self):
        self.recorded = 0
        self.synced = 0

    def record(self, stream=None):
        self.recorded += 1

    def synchronize(self):
        self.synced += 1


def _ring():
    r = kernels._LadderRing.__new__(kernels._LadderRing)
    r.dev = None
    r.blocks = [_Block() for _ in range(kernels._LadderRing.N)]
    r.events = [_Event() for _ in range(kernels._LadderRing.N)]
    r.pending = [None] * kernels._LadderRing.N
    r.next = 0
    r.gen = 0
    return r


def test_backward_settles_its_own_forward():
    r = _ring()
    tok, words = r.take(3, "qEHVI posterior root")
    assert len(words) == 3
    r.blocks[tok[0]].words[3] = 1e-6  # member 1 jittered
    with pytest.warns(NumericalWarning, match="1.0e-06"):
        r.settle(tok)
    assert r.pending[tok[0]] is None and r.events[tok[0]].synced == 1
    r.settle(tok)  # settled once: nothing more


def test_stale_token_does_not_settle_a_newer_forward():
    r = _ring()
    tok0, _ = r.take(2, "a")
    for _ in range(kernels._LadderRing.N):  # the ring comes round: tok0's block reused
        tok, _ = r.take(2, "b")
    assert tok[0] == tok0[0] and tok[1] != tok0[1]
    r.blocks[tok[0]].words[0] = 1.0  # the NEWER forward failed
    r.settle(tok0)  # the old token: no read, no raise
    assert r.pending[tok[0]] is not None
    with pytest.raises(NotPSDError, match="b"):
        r.settle(tok)


def test_block_coming_round_reports_the_forward_left_pending():
    r = _ring()
    tok0, _ = r.take(1, "first")
    r.blocks[tok0[0]].words[0] = 1.0  # its backward never ran
    for _ in range(kernels._LadderRing.N - 1):
        r.take(1, "later")
    with pytest.raises(NotPSDError, match="first"):
        r.take(1, "wraps")  # the reuse of tok0's block reads it first
    assert r.pending[tok0[0]] is None


def test_settle_all_oldest_first_and_member_order():
    r = _ring()
    t1, _ = r.take(2, "one")
    t2, _ = r.take(2, "two")
    r.blocks[t1[0]].words[1] = 1e-8
    r.blocks[t2[0]].words[2] = 1.0  # member 1 of the second forward failed
    with warnings.catch_warnings(record=True) as ws:
        warnings.simplefilter("always")
        with pytest.raises(NotPSDError, match="two"):
            r.settle_all()
    assert any(issubclass(w.category, NumericalWarning) for w in ws)  # "one" reported first
    assert all(p is None for p in r.pending)
