"""Environments: the OthelloGameNew drop-in (bitboard engine behind the C ABI) and the
copy-on-step TicTacToe of config #1."""
