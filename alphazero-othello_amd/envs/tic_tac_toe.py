"""TicTacToe (reference envs/tic_tac_toe.py:6-72) for config #1 (CPU plumbing).

One intended deviation: get_next_state copies the state before placing the stone.  The
reference mutates in place (:25-29), so MCTS children alias their parent's array
(MCTS_model.py:149) and self-play with tree reuse never finishes; every
other method is the reference's rule set.
"""
import numpy as np

from .game import Game


class TicTacToe(Game):

    def __init__(self):
        self.row_count = 3
        self.column_count = 3
        self._action_size = self.row_count * self.column_count
        self._state_size = self._action_size

    def get_initial_state(self):
        return np.zeros((self.row_count, self.column_count))

    @property
    def action_size(self):
        return self._action_size

    @property
    def state_size(self):
        return self._state_size

    def get_next_state(self, state, action, player):
        state = np.array(state, copy=True)
        state[action // self.column_count, action % self.column_count] = player
        return state

    def get_valid_moves(self, state, player):
        return (state.reshape(-1) == 0).astype(np.uint8)

    def check_win(self, state, action):
        """+1/-1 if the stone just placed at `action` completes a line, else 0
        (reference :34-56)."""
        row, column = action // self.column_count, action % self.column_count
        player = state[row, column]
        n = self.row_count
        lines = (np.sum(state[row, :]), np.sum(state[:, column]), np.sum(np.diag(state)),
                 np.sum(np.diag(np.flipud(state))))
        if any(s == player * n for s in lines):
            return player
        return 0

    def get_value_and_terminated(self, state, action, current_player):
        winner = self.check_win(state, action)
        if winner != 0:
            return winner * current_player, True
        if np.sum(self.get_valid_moves(state, current_player)) == 0:
            return 0, True
        return 0, False

    def get_opponent(self, player):
        return -player
