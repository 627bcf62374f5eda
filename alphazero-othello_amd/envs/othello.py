"""OthelloGameNew drop-in backed by the native bitboard engine (C ABI, libaz_othello.so).

Reference: envs/othello.py:309-498 (`OthelloGameNew`) and :129-220 (`_BitBoard`).  Same
class names, constructor, properties, method signatures, return dtypes and exceptions, so
MCTS_model.py, self_play_worker.py, train.py and eval.py use it unchanged.  What changed
is the engine underneath: every rule evaluation is one call into the C ABI (reentrant,
GIL released by ctypes), instead of the reference's per-call 64-step Python conversion
loops and 8 x 6 NumPy shift fills.

State at the API edge stays the reference's int8 (8,8) absolute-colour array (+1 moves
first).  Internally bit r*8+c <-> square (r, c) (the `_BitBoard` layout, :202-212); the
reference's OthelloGameNew additionally rotates by 180 degrees (:336-356), which the static
helpers below keep for callers that use them directly.
"""
import numpy as np

import az_native as nat

from .game import Game

_BITS = np.uint64(1) << np.arange(64, dtype=np.uint64)


def _mask_to_valid(mask):
    """uint64 placement mask -> uint8[65] valid vector, [64] set iff no placement
    (envs/othello.py:401-411)."""
    valid = np.zeros(65, np.uint8)
    m = int(mask)
    if m == 0:
        valid[64] = 1
    else:
        valid[:64] = (np.uint64(m) & _BITS) != 0
    return valid


class _BitBoard:
    """Bitboard with `black` = side to move (reference envs/othello.py:129-220)."""

    __slots__ = ("black", "white", "perspective")

    def __init__(self):
        self.black = np.uint64(0x0000000810000000)
        self.white = np.uint64(0x0000001008000000)
        self.perspective = 1

    @staticmethod
    def _lsb(mask):
        m = int(mask)
        return (m & -m).bit_length() - 1

    def _legal_moves(self, own, opp):
        return np.uint64(nat.legal_cpu(np.array([own]), np.array([opp]))[0])

    def valid_mask(self):
        return self._legal_moves(self.black, self.white)

    def make_move(self, action):
        """Play `action` (0-63) for the side to move, 64 = pass; like the reference there is
        no legality check (an unbounded placement captures nothing)."""
        o, p = nat.make_move_cpu(np.array([self.black]), np.array([self.white]),
                                 np.array([action]))
        self.black, self.white = np.uint64(o[0]), np.uint64(p[0])
        self.perspective *= -1

    def to_numpy(self):
        black, white = ((self.black, self.white) if self.perspective == 1 else
                        (self.white, self.black))
        return nat.unpack_np(np.array([black]), np.array([white]), 1)[0]

    def score(self):
        return int(int(self.black).bit_count() - int(self.white).bit_count())


def popcount(x):
    return np.vectorize(lambda v: int(int(v).bit_count()), otypes=[int])(x)


class OthelloGameNew(Game):
    """Same public interface as the reference class, backed by the native engine."""

    square_content = {-1: "X", 0: "-", 1: "O"}

    @staticmethod
    def get_square_piece(piece):
        return OthelloGameNew.square_content[piece]

    def __init__(self, n):
        assert n == 8, "Bitboard engine supports only standard 8×8 Othello"
        self.n = n
        self._state_size = n * n
        self._action_size = self._state_size + 1

    @property
    def action_size(self):
        return self._action_size

    @property
    def state_size(self):
        return self._state_size

    # ---- the reference's 180-degree-rotated bit helpers (envs/othello.py:336-388) ----
    @staticmethod
    def _idx_to_bit(idx):
        row, col = divmod(idx, 8)
        return (7 - row) * 8 + (7 - col)

    @staticmethod
    def _bit_to_idx(bit):
        row, col = divmod(bit, 8)
        return (7 - row) * 8 + (7 - col)

    @staticmethod
    def _np_to_bitboards(state, player):
        own, opp = nat.pack_np(state, player)
        # row-major bit r*8+c -> the reference's rotated bit 63-(r*8+c): a bit reversal
        return (np.uint64(int(f"{int(own[0]):064b}"[::-1], 2)),
                np.uint64(int(f"{int(opp[0]):064b}"[::-1], 2)))

    @staticmethod
    def _bitboards_to_np(black, white):
        b = int(f"{int(black):064b}"[::-1], 2)
        w = int(f"{int(white):064b}"[::-1], 2)
        return nat.unpack_np(np.array([b], np.uint64), np.array([w], np.uint64), 1)[0]

    # ---- rows of the Game interface ----------------------------------------------
    @staticmethod
    def _bb(state, player):
        own, opp = nat.pack_np(state, player)
        return own, opp

    def get_initial_state(self):
        s = np.zeros((8, 8), np.int8)
        s[3, 4] = s[4, 3] = 1
        s[3, 3] = s[4, 4] = -1
        return s

    def get_valid_moves(self, state, player):
        own, opp = self._bb(state, player)
        return _mask_to_valid(nat.legal_cpu(own, opp)[0])

    def get_next_state(self, state, action, player):
        action = int(action)
        if action == self._state_size:  # pass: copy, no legality check (:415-416)
            return np.array(state, copy=True)
        if not 0 <= action < self._state_size:
            raise ValueError(f"Illegal move: {action}")
        own, opp = self._bb(state, player)
        o, p, _, st = nat.step_cpu(own, opp, np.array([action]), raise_illegal=False)
        if st[0] & nat.AZ_FLAG_ILLEGAL:
            raise ValueError(f"Illegal move: {action}")  # envs/othello.py:419-421
        return nat.unpack_np(o, p, -player)[0]

    def get_value_and_terminated(self, state, action, player):
        # `action` is ignored, as in the reference (:435-454)
        own, opp = self._bb(state, player)
        if int(nat.legal_cpu(own, opp)[0]) or int(nat.legal_cpu(opp, own)[0]):
            return 0, False
        diff = int(own[0]).bit_count() - int(opp[0]).bit_count()
        return (1 if diff > 0 else (-1 if diff < 0 else 0)), True

    def get_score(self, state, player):
        return int(np.sum(state == player) - np.sum(state == -player))

    def get_opponent(self, player):
        return -player

    def print_board(self, state, player, ply=None):
        """The reference's text rendering (envs/othello.py:459-498)."""
        lines = ["  a b c d e f g h"]
        to_ch = OthelloGameNew.square_content
        for r in range(8):
            row = [str(r + 1)]
            for c in range(8):
                row.append(to_ch[-int(state[r, c])])
            lines.append(" ".join(row))
        print("\n".join(lines))


def get_random_symmetry(state, pi):
    """One random dihedral transform of (state, pi) for training augmentation
    (reference envs/othello.py:501-526; same np.random draw order)."""
    n = state.shape[-1]
    k = np.random.randint(4)
    flip = np.random.rand() < 0.5
    s = np.rot90(state, k, axes=(-2, -1))
    pb = np.rot90(pi[:-1].reshape(n, n), k)
    if flip:
        s = np.fliplr(s)
        pb = np.fliplr(pb)
    if s.ndim == 2:
        s = s[None, :, :]
    s = np.ascontiguousarray(s, dtype=np.float32)
    pi_out = np.concatenate([pb.ravel(), pi[-1:]]).astype(np.float32, copy=False)
    return s, pi_out
