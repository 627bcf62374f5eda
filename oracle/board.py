"""TEST INFRASTRUCTURE ONLY — numpy/ctypes wrapper of oracle/oth_oracle.c.

Restates the reference bitboard engine (envs/othello.py:112-220) and the
OthelloGameNew array API (envs/othello.py:309-457) for the parity checks.
"""
import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboth_oracle.so")
_lib = None


def build():
    subprocess.check_call(["make", "-s", "-C", _HERE])


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        L = ctypes.CDLL(_SO)
        u64, i64, i32 = ctypes.c_uint64, ctypes.c_int64, ctypes.c_int
        P = ctypes.c_void_p
        L.oracle_legal.argtypes = [u64, u64]
        L.oracle_legal.restype = u64
        L.oracle_make_move.argtypes = [u64, u64, i32, P, P]
        L.oracle_make_move.restype = None
        L.oracle_step.argtypes = [P, P, P, P, P, P, P, i64]
        L.oracle_step.restype = i64
        L.oracle_legal_batch.argtypes = [P, P, P, i64]
        L.oracle_legal_batch.restype = None
        L.oracle_rollout.argtypes = [u64, u64, u64]
        L.oracle_rollout.restype = i32
        _lib = L
    return _lib


def _p(a):
    return a.ctypes.data_as(ctypes.c_void_p)


def legal(own, opp):
    return int(lib().oracle_legal(int(own), int(opp)))


def make_move(own, opp, action):
    a, b = ctypes.c_uint64(), ctypes.c_uint64()
    lib().oracle_make_move(int(own), int(opp), int(action), ctypes.byref(a), ctypes.byref(b))
    return a.value, b.value


def step_batch(own, opp, act):
    own = np.ascontiguousarray(own, np.uint64)
    opp = np.ascontiguousarray(opp, np.uint64)
    act = np.ascontiguousarray(act, np.uint8)
    n = len(own)
    o, p, lg = (np.empty(n, np.uint64) for _ in range(3))
    st = np.empty(n, np.uint16)
    bad = lib().oracle_step(_p(own), _p(opp), _p(act), _p(o), _p(p), _p(lg), _p(st), n)
    return o, p, lg, st, int(bad)


def legal_batch(own, opp):
    own = np.ascontiguousarray(own, np.uint64)
    opp = np.ascontiguousarray(opp, np.uint64)
    out = np.empty(len(own), np.uint64)
    lib().oracle_legal_batch(_p(own), _p(opp), _p(out), len(own))
    return out


_W = np.uint64(1) << np.arange(64, dtype=np.uint64)


def to_bitboards(state, player):
    """(8,8) absolute-colour state -> (own, opp) with own = stones of `player`."""
    flat = np.asarray(state).reshape(-1)
    own = int(np.bitwise_or.reduce(np.where(flat == player, _W, np.uint64(0))))
    opp = int(np.bitwise_or.reduce(np.where(flat == -player, _W, np.uint64(0))))
    return own, opp


def to_state(own, opp, player):
    bits_o = (np.uint64(own) >> np.arange(64, dtype=np.uint64)) & np.uint64(1)
    bits_p = (np.uint64(opp) >> np.arange(64, dtype=np.uint64)) & np.uint64(1)
    s = np.where(bits_o == 1, player, np.where(bits_p == 1, -player, 0)).astype(np.int8)
    return s.reshape(8, 8)


def popc(x):
    return bin(int(x)).count("1")


class OracleGame:
    """The OthelloGameNew array API (envs/othello.py:309-457) restated on the oracle."""

    action_size = 65
    state_size = 64
    n = 8

    def get_initial_state(self):
        s = np.zeros((8, 8), np.int8)
        s[3, 4] = s[4, 3] = 1
        s[3, 3] = s[4, 4] = -1
        return s

    def get_valid_moves(self, state, player):
        own, opp = to_bitboards(state, player)
        m = legal(own, opp)
        v = np.zeros(65, np.uint8)
        if m == 0:
            v[64] = 1
        else:
            v[:64] = ((np.uint64(m) >> np.arange(64, dtype=np.uint64)) & np.uint64(1))
        return v

    def get_next_state(self, state, action, player):
        if action == 64:
            return np.array(state, copy=True)
        own, opp = to_bitboards(state, player)
        if not (legal(own, opp) >> int(action)) & 1:
            raise ValueError(f"Illegal move: {action}")
        no, np_ = make_move(own, opp, int(action))
        return to_state(no, np_, -player)

    def get_value_and_terminated(self, state, action, player):
        own, opp = to_bitboards(state, player)
        if legal(own, opp) or legal(opp, own):
            return 0, False
        d = popc(own) - popc(opp)
        return (1 if d > 0 else (-1 if d < 0 else 0)), True

    def get_score(self, state, player):
        own, opp = to_bitboards(state, player)
        return popc(own) - popc(opp)

    def get_opponent(self, player):
        return -player
