"""Replay of the np.random draws the reference made while the golden MCTS / self-play
vectors were recorded (tests/golden/make_goldens.py RngRecorder), for the drop-in classes
and for the engine's injected-RNG streams."""
import numpy as np


def case_log(d, c):
    lo, hi = int(d["log_offsets"][c]), int(d["log_offsets"][c + 1])
    nlo, nhi = int(d["noise_offsets"][c]), int(d["noise_offsets"][c + 1])
    return d["log_kind"][lo:hi], d["log_a"][lo:hi], d["log_b"][lo:hi], d["noise"][nlo:nhi]


def engine_streams(kinds, a, b, noise):
    """Injected-stream form: the Dirichlet vectors in order, and one uniform per
    choice draw (tie break -> (j + 0.5) / k so floor(u * k) = j; action sample -> u)."""
    us = []
    for k, x, y in zip(kinds, a, b):
        if k == 1:
            us.append((int(y) + 0.5) / int(x))
        elif k == 2:
            us.append(float(x))
    return np.asarray(noise, np.float64).reshape(-1, 65), np.asarray(us, np.float64)


class ReplayNpRandom:
    """Context manager: np.random.dirichlet / np.random.choice return the recorded draws."""

    def __init__(self, kinds, a, b, noise):
        self.kinds, self.a, self.b, self.noise = list(kinds), list(a), list(b), noise
        self.i = 0

    def __enter__(self):
        self._dir, self._choice = np.random.dirichlet, np.random.choice
        me = self

        def dirichlet(alpha, size=None):
            assert me.kinds[me.i] == 0, f"draw {me.i}: dirichlet not expected"
            v = np.array(me.noise[int(me.a[me.i])], np.float64)
            me.i += 1
            return v

        def choice(arr, size=None, replace=True, p=None):
            k = me.kinds[me.i]
            if p is not None:
                assert k == 2, f"draw {me.i}: choice(p) not expected"
                u = float(me.a[me.i])
                cdf = np.asarray(p, np.float64).cumsum()
                cdf /= cdf[-1]
                me.i += 1
                return int(cdf.searchsorted(u, side="right"))
            assert k == 1, f"draw {me.i}: tie choice not expected"
            arr = np.asarray(arr)
            assert len(arr) == int(me.a[me.i])
            r = arr[int(me.b[me.i])]
            me.i += 1
            return r

        np.random.dirichlet, np.random.choice = dirichlet, choice
        return self

    def __exit__(self, *exc):
        np.random.dirichlet, np.random.choice = self._dir, self._choice
