"""The abstract environment interface of the reference (envs/game.py:5-57)."""
from abc import ABC, abstractmethod


class Game(ABC):

    @abstractmethod
    def get_initial_state(self):
        """Initial state of the board."""

    @abstractmethod
    def get_valid_moves(self, state, player):
        """Binary vector of valid moves for `player`."""

    @property
    @abstractmethod
    def action_size(self):
        """Number of actions."""

    @property
    @abstractmethod
    def state_size(self):
        """Number of board cells."""

    @abstractmethod
    def get_next_state(self, state, action, player):
        """Next state after `player` plays `action`."""

    @abstractmethod
    def get_value_and_terminated(self, state, action, player):
        """(value from `player`'s view, game over?)."""

    @abstractmethod
    def get_opponent(self, player):
        """Opponent of `player`."""
