"""libmanette_host bookkeeping (mh_book) == the Python Bookkeeper (pinned to the reference's golden
host-loop vectors in test_host_cpu.py) on random macro-steps, and == G1 directly. CPU only."""
import os

import numpy as np
import pytest

from manette_amd.bookkeeping import Bookkeeper, NativeBook

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


@pytest.mark.parametrize('E,A,tab', [(4, 6, [0]), (32, 4, list(range(11))), (7, 18, [0, 2, 4, 6, 8, 10])])
def test_native_book_matches_python(E, A, tab):
    rs = np.random.RandomState(E)
    py = Bookkeeper(E, A, tab)
    nb = NativeBook(E, A, tab)
    gp = gn = 123
    for u in range(6):
        py.new_update()
        nb.new_update()
        for t in range(5):
            a = rs.randint(0, A, E).astype(np.int32)
            r = rs.randint(0, len(tab), E).astype(np.int32)
            reward = rs.choice([-3.0, -1.0, 0.0, 0.5, 1.0, 2.0], E).astype(np.float32)
            over = (rs.rand(E) < 0.2).astype(np.float32)
            r1, m1 = np.zeros(E, np.float32), np.zeros(E, np.float32)
            r2, m2 = np.zeros(E, np.float32), np.zeros(E, np.float32)
            gp = py.step(gp, a, r, reward, over, r1, m1)
            gn = nb.step(gn, a, r, reward, over, r2, m2)
            assert gp == gn
            np.testing.assert_array_equal(r1, r2)
            np.testing.assert_array_equal(m1, m2)
        for x, y in zip(py.histograms(), nb.histograms()):
            np.testing.assert_array_equal(x, y)
        assert nb.nb_actions == py.nb_actions
    assert py.episodes == nb.episodes
    assert py.total_rewards == nb.total_rewards and py.total_steps == nb.total_steps


def test_native_book_rejects_bad_index():
    from manette_amd import _lib
    nb = NativeBook(2, 3, [0, 1])
    z = np.zeros(2, np.float32)
    with pytest.raises(_lib.MTError):
        nb.step(0, np.array([0, 3], np.int32), np.array([0, 0], np.int32), z, z, z.copy(), z.copy())
