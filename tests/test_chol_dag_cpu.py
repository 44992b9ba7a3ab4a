"""Host logic of the persistent Cholesky DAG (csrc/chol_dag.hip): the task
queue is a topological order of the dependencies the kernel waits on (the
no-deadlock argument of the queue), every tile row is covered exactly once per
step, and the queue holds the expected task set.  Runs on the CPU: the library
builds the queue without touching a device."""
import ctypes

import numpy as np
import pytest

T_CRIT, T_TRSM, T_COLUPD, T_XSTEP, T_AINV = 0, 1, 2, 3, 4


def _queue(T, ainv=False):
    from botorch_amd._lib import lib
    fn = lib().bo_chol_dag_tasks_ainv if ainv else lib().bo_chol_dag_tasks
    n = fn(T, None, 0)
    buf = np.zeros(4 * n, dtype=np.int32)
    m = fn(T, buf.ctypes.data_as(ctypes.c_void_p), n)
    assert m == n
    q = buf.reshape(n, 4)
    return [(int(x) & 0xFF, (int(x) >> 8) & 0xFF, int(k), int(j), int(w) & 0xFFFF, int(w) >> 16,
             max(1, int(x) >> 16)) for x, k, j, w in q]


@pytest.mark.parametrize("ainv", [False, True])
@pytest.mark.parametrize("T", [1, 2, 3, 5, 16, 64])
def test_queue_is_topological_and_complete(T, ainv):
    """ainv: the queue with the A^{-1} = X^T X tasks (bo_cholesky_inverse_ainv):
    each reads X tiles only once final (X_Ki final with X_{ke-1,i}), and every
    lower tile (i, j) takes its contributions K = i .. T - 1 in increasing K."""
    q = _queue(T, ainv)
    L = set()                 # final L tiles
    A = {}                    # (i, j) -> updates applied
    X = {}                    # (i, j) -> updates applied to X's accumulator
    Xd = set()                # finalised X tiles (k > j)
    Ai = {}                   # (i, j) -> A^{-1} contributions applied
    assert any(t[0] == T_AINV for t in q) == ainv

    def x_final(kk, jj):
        return (kk, jj) in Xd or (kk == jj and (jj, jj) in L)

    for type_, fin, k, j, i0, i1, nk in q:
        if type_ == T_AINV:
            ke = k + nk
            assert all(x_final(kk, j) for kk in range(max(k, j), ke))
            for i in range(i0, i1):
                assert j <= i < ke
                assert all(x_final(kk, i) for kk in range(max(k, i), ke))
                assert Ai.get((i, j), 0) == max(k, i) - i
                Ai[(i, j)] = ke - i
            continue
        if type_ == T_CRIT:
            if k > 0:
                assert A.get((k, k - 1), 0) >= k - 1 and (k - 1, k - 1) in L
                assert A.get((k, k), 0) >= k - 1
                L.add((k, k - 1))
                A[(k, k)] = k
            L.add((k, k))
        elif type_ == T_TRSM:
            assert (k, k) in L
            for i in range(i0, i1):
                assert A.get((i, k), 0) >= k and (i, k) not in L
                L.add((i, k))
        elif type_ == T_COLUPD:  # steps k .. k + nk - 1 (nk > 1: a batched update)
            assert all((j, kk) in L for kk in range(k, k + nk))
            for i in range(i0, i1):
                assert all((i, kk) in L for kk in range(k, k + nk)) and A.get((i, j), 0) == k
                A[(i, j)] = k + nk
        elif nk > 1:  # XSTEP, batched: steps k .. k + nk - 1 on far rows
            assert all((kk, j) in Xd or (kk == j and (j, j) in L) for kk in range(k, k + nk))
            for i in range(i0, i1):
                assert i >= k + nk
                assert all((i, kk) in L for kk in range(k, k + nk)) and X.get((i, j), 0) == k - j
                X[(i, j)] = k + nk - j
        else:
            if k == j:
                assert (k, k) in L
            elif fin:
                assert X.get((k, j), 0) == k - j and (k, k) in L
                Xd.add((k, j))
            else:
                assert (k, j) in Xd
            for i in range(i0, i1):
                assert (i, k) in L and X.get((i, j), 0) == k - j
                X[(i, j)] = k - j + 1
    # complete: every L tile final, every tile took all its updates, every X
    # tile below the diagonal finalised
    assert L == {(i, j) for i in range(T) for j in range(i + 1)}
    for i in range(T):
        for j in range(i + 1):
            assert A.get((i, j), 0) == j
    assert Xd == {(k, j) for k in range(T) for j in range(k)}
    assert all(X[(i, j)] == i - j for i in range(T) for j in range(i))
    if ainv:
        assert Ai == {(i, j): T - i for i in range(T) for j in range(i + 1)}
